// generation_rows_f64.hip — double instantiations of the short-row hot kernel
// (generation_rows.hpp; split per genome type so hipcc runs them in parallel).
#include "generation_rows.hpp"

namespace dm {

void launch_gen_rows_f64(const GenArgs& a, const PairPlan* plans, int ec, int num_cus,
                        hipStream_t s) {
    launch_rows_t<double>(a, plans, ec, num_cus, s);
}

}  // namespace dm
