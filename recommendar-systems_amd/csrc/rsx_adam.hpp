// rsx_adam.hpp — torch.optim.Adam's single-tensor update, element by element
// (reference src/common/trainer.py:133,238 builds torch.optim.Adam): shared by the
// SpMM ADAM epilogue (spmm.hip) and the multi-tensor launch (smore_fuse.hip).
#pragma once
#include <cmath>

#include "rsx_common.hpp"

namespace rsx {

struct AdamConst {
    float lr, omb1, b2, omb2, eps, wd, step_size, bc2_sqrt;
};

__device__ __forceinline__ AdamConst adam_const(const rsx_adam& a) {
    AdamConst c;
    const int64_t step = a.step_dev ? *a.step_dev : a.step;
    // torch.optim.Adam (_single_tensor_adam): bias corrections in double, the
    // tensor ops in f32 with the scalars rounded to f32.
    const double bc1 = 1.0 - pow((double)a.beta1, (double)step);
    const double bc2 = 1.0 - pow((double)a.beta2, (double)step);
    c.lr = a.lr;
    c.omb1 = (float)(1.0 - (double)a.beta1);
    c.b2 = a.beta2;
    c.omb2 = (float)(1.0 - (double)a.beta2);
    c.eps = a.eps;
    c.wd = a.weight_decay;
    c.step_size = (float)((double)a.lr / bc1);
    c.bc2_sqrt = (float)sqrt(bc2);
    return c;
}

__device__ __forceinline__ float adam_elem(const AdamConst& c, float& p, float& m, float& v, float g) {
    if (c.wd != 0.f) g = g + c.wd * p;
    m = m + c.omb1 * (g - m);                 // exp_avg.lerp_(grad, 1 - beta1)
    v = v * c.b2 + (c.omb2 * g) * g;          // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
    const float denom = sqrtf(v) / c.bc2_sqrt + c.eps;
    p = p + (-c.step_size) * m / denom;       // param.addcdiv_(exp_avg, denom, -step_size)
    return g;
}

}  // namespace rsx
