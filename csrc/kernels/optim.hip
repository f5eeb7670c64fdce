// Multi-replica fused SGD (K10): torch.optim.SGD(momentum, weight_decay) semantics on the
// flat [G, P] buffers of all concurrently-training clients in ONE launch, with per-client
// learning rate (benign lr / poison lr with the MultiStepLR schedule), per-client
// "fresh optimizer" flag (momentum buffer := d_p on its first step), per-client activity
// mask and the FoolsGold raw-gradient accumulation (image_train.py:94-100), all in the same
// pass over the parameters.
#include "common.hpp"
#include <algorithm>

namespace {

__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ params, long long p_gstride,
                                                  const float* __restrict__ grads, float* __restrict__ mom,
                                                  const float* __restrict__ lr, const int* __restrict__ first,
                                                  const int* __restrict__ active, float momentum, float wd,
                                                  float* __restrict__ fg, int P) {
  const int g = blockIdx.y;
  if (!active[g]) return;
  const float l = lr[g];
  const bool f = first[g] != 0;
  float* p = params + (long long)g * p_gstride;
  const float* gr = grads + (long long)g * P;
  float* m = mom + (long long)g * P;
  float* fa = fg ? fg + (long long)g * P : nullptr;
  for (int i4 = blockIdx.x * blockDim.x + threadIdx.x; i4 < P / 4; i4 += gridDim.x * blockDim.x) {
    const int i = i4 * 4;
    float4 pv = *(float4*)(p + i);
    const float4 gv = *(const float4*)(gr + i);
    float4 mv = f ? make_float4(0, 0, 0, 0) : *(const float4*)(m + i);
    if (fa) {
      float4 a = *(float4*)(fa + i);
      a.x += gv.x; a.y += gv.y; a.z += gv.z; a.w += gv.w;
      *(float4*)(fa + i) = a;
    }
    float* pp = (float*)&pv;
    const float* gp = (const float*)&gv;
    float* mp = (float*)&mv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = gp[e] + wd * pp[e];
      mp[e] = f ? d : momentum * mp[e] + d;
      pp[e] -= l * mp[e];
    }
    *(float4*)(p + i) = pv;
    *(float4*)(m + i) = mv;
  }
}

}  // namespace

DBA_EXPORT int dba_sgd_step(float* params, long long p_gstride, const float* grads, float* mom, const float* lr,
                            const int* first, const int* active, float momentum, float wd, float* fg,
                            int G, int P, void* stream) {
  const int blocks = std::max(1, std::min(1024, (P / 4 + 255) / 256));
  hipLaunchKernelGGL(sgd_kernel, dim3(blocks, G), dim3(256), 0, (hipStream_t)stream, params, p_gstride, grads, mom, lr,
                     first, active, momentum, wd, fg, P);
  DBA_LAUNCH_CHECK();
}
