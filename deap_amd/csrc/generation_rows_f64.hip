// generation_rows_f64.hip — double instantiations of the whole-row hot
// kernel (generation_rows.hpp).
#include "generation_rows.hpp"

namespace dm {

template <int NCH, int CX, int MUT>
static void launch_e(const GenArgs& a, int ec, dim3 grid, hipStream_t s) {
    if (ec == EC_RAST)
        gen_rows_kernel<double, NCH, CX, MUT, EC_RAST><<<grid, 256, 0, s>>>(a);
    else if (ec == EC_ROSEN)
        gen_rows_kernel<double, NCH, CX, MUT, EC_ROSEN><<<grid, 256, 0, s>>>(a);
    else if (ec_single(ec))
        gen_rows_kernel<double, NCH, CX, MUT, EC_SUM><<<grid, 256, 0, s>>>(a);
    else
        gen_rows_kernel<double, NCH, CX, MUT, EC_NONE><<<grid, 256, 0, s>>>(a);
}
template <int NCH>
static void launch_ops(const GenArgs& a, int ec, dim3 grid, hipStream_t s) {
    const bool mg = a.mut == DM_MUT_GAUSSIAN;
    switch (a.cx) {
        case DM_CX_BLEND:
            mg ? launch_e<NCH, DM_CX_BLEND, DM_MUT_GAUSSIAN>(a, ec, grid, s)
               : launch_e<NCH, DM_CX_BLEND, DM_MUT_NONE>(a, ec, grid, s);
            break;
        case DM_CX_TWOPOINT:
            mg ? launch_e<NCH, DM_CX_TWOPOINT, DM_MUT_GAUSSIAN>(a, ec, grid, s)
               : launch_e<NCH, DM_CX_TWOPOINT, DM_MUT_NONE>(a, ec, grid, s);
            break;
        default:
            mg ? launch_e<NCH, DM_CX_NONE, DM_MUT_GAUSSIAN>(a, ec, grid, s)
               : launch_e<NCH, DM_CX_NONE, DM_MUT_NONE>(a, ec, grid, s);
    }
}
void launch_gen_rows_f64(const GenArgs& a, int ec, int nch, dim3 grid, hipStream_t s) {
    if (nch <= 2)
        launch_ops<2>(a, ec, grid, s);
    else
        launch_ops<4>(a, ec, grid, s);
}

}  // namespace dm
