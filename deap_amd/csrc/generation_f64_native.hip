// generation_f64_native.hip — double-genome instantiations of the fused
// generation kernel, native mode (split per file so hipcc runs in parallel).
#include "generation.hpp"

namespace dm {

template <int G, int CX, int MUT>
static void launch_g(const GenArgs& a, int ec, dim3 grid, hipStream_t s) {
    if (G == 64 && ec == EC_RAST)
        gen_float_kernel<double, G, CX, MUT, EC_RAST, false><<<grid, 256, 0, s>>>(a);
    else if (G == 64 && ec == EC_ROSEN)
        gen_float_kernel<double, G, CX, MUT, EC_ROSEN, false><<<grid, 256, 0, s>>>(a);
    else if (ec_single(ec))
        gen_float_kernel<double, G, CX, MUT, EC_SUM, false><<<grid, 256, 0, s>>>(a);
    else if (ec == EC_MO)
        gen_float_kernel<double, G, CX, MUT, EC_MO, false><<<grid, 256, 0, s>>>(a);
    else
        gen_float_kernel<double, G, CX, MUT, EC_NONE, false><<<grid, 256, 0, s>>>(a);
}
template <int G>
static void launch_ops(const GenArgs& a, int ec, dim3 grid, hipStream_t s) {
    const bool mg = a.mut == DM_MUT_GAUSSIAN;
    switch (a.cx) {
        case DM_CX_BLEND:
            mg ? launch_g<G, DM_CX_BLEND, DM_MUT_GAUSSIAN>(a, ec, grid, s)
               : launch_g<G, DM_CX_BLEND, DM_MUT_NONE>(a, ec, grid, s);
            break;
        case DM_CX_TWOPOINT:
            mg ? launch_g<G, DM_CX_TWOPOINT, DM_MUT_GAUSSIAN>(a, ec, grid, s)
               : launch_g<G, DM_CX_TWOPOINT, DM_MUT_NONE>(a, ec, grid, s);
            break;
        default:
            mg ? launch_g<G, DM_CX_NONE, DM_MUT_GAUSSIAN>(a, ec, grid, s)
               : launch_g<G, DM_CX_NONE, DM_MUT_NONE>(a, ec, grid, s);
    }
}
void launch_gen_f64_native(const GenArgs& a, int ec, int G, dim3 grid, hipStream_t s) {
    switch (G) {
        case 4: launch_ops<4>(a, ec, grid, s); break;
        case 16: launch_ops<16>(a, ec, grid, s); break;
        default: launch_ops<64>(a, ec, grid, s); break;
    }
}

}  // namespace dm
