// generation_pipe_long.hip -- the rolling-pipeline hot kernel (generation_pipe.hpp)
// for float rows of more than 1,024 genes: the chunk count is read at run time
// (NCH = 0), so one instantiation per operator set covers every row length.
#include "generation_pipe.hpp"

namespace dm {

void launch_gen_pipe_long(const PipeArgs& a, bool f64, int ec, int cx, int mut, int num_cus,
                          hipStream_t s) {
    if (f64)
        launch_pipe_ops<double, 0>(a, ec, cx, mut, num_cus, s);
    else
        launch_pipe_ops<float, 0>(a, ec, cx, mut, num_cus, s);
}

}  // namespace dm
