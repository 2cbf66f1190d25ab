// generation_pipe_f32.hip — float instantiations of the rolling-pipeline hot
// kernel (generation_pipe.hpp).
#include "generation_pipe.hpp"

namespace dm {

void launch_gen_pipe_f32(const PipeArgs& a, int ec, int cx, int mut, int nch, int num_cus,
                         hipStream_t s) {
    if (nch == 0)
        launch_gen_pipe_long(a, false, ec, cx, mut, num_cus, s);
    else if (nch <= 2)
        launch_pipe_ops<float, 2>(a, ec, cx, mut, num_cus, s);
    else
        launch_pipe_ops<float, 4>(a, ec, cx, mut, num_cus, s);
}

}  // namespace dm
