// generation_bits.hip — packed-bit instantiations of the fused generation kernel.
#include "generation.hpp"

namespace dm {

template <int G, int CX, int MUT, bool RP>
static void launch_m(const GenArgs& a, int ec, dim3 grid, hipStream_t s) {
    if (ec != EC_NONE)
        gen_bits_kernel<G, CX, MUT, EC_SUM, RP><<<grid, 256, 0, s>>>(a);
    else
        gen_bits_kernel<G, CX, MUT, EC_NONE, RP><<<grid, 256, 0, s>>>(a);
}
template <int G, int CX, int MUT>
static void launch_g(const GenArgs& a, int ec, dim3 grid, hipStream_t s) {
    if (a.mode == DM_RNG_NATIVE)
        launch_m<G, CX, MUT, false>(a, ec, grid, s);
    else
        launch_m<G, CX, MUT, true>(a, ec, grid, s);
}
template <int G>
static void launch_ops(const GenArgs& a, int ec, dim3 grid, hipStream_t s) {
    const bool mf = a.mut == DM_MUT_FLIPBIT;
    if (a.cx == DM_CX_TWOPOINT)
        mf ? launch_g<G, DM_CX_TWOPOINT, DM_MUT_FLIPBIT>(a, ec, grid, s)
           : launch_g<G, DM_CX_TWOPOINT, DM_MUT_NONE>(a, ec, grid, s);
    else
        mf ? launch_g<G, DM_CX_NONE, DM_MUT_FLIPBIT>(a, ec, grid, s)
           : launch_g<G, DM_CX_NONE, DM_MUT_NONE>(a, ec, grid, s);
}
void launch_gen_bits(const GenArgs& a, int ec, int G, dim3 grid, hipStream_t s) {
    switch (G) {
        case 2: launch_ops<2>(a, ec, grid, s); break;
        case 8: launch_ops<8>(a, ec, grid, s); break;
        default: launch_ops<64>(a, ec, grid, s); break;
    }
}

}  // namespace dm
