// Device-resident windowing of trajectories (common/data_creator.py:48-78, DataCreator.create_data):
// out[b][c][t][hw] = u[b][c][steps[b] + offset + t][hw] for t < tw (offset -tw: inputs, 0: labels).
// One gather per batch replaces the reference's per-sample slicing + torch.cat + host->device copy.
// HBM-bound copy: float4 per thread along the contiguous (H*W) plane.
#include "nps_common.hpp"

namespace {

template <bool VEC>
__global__ void gather_windows_kernel(const float* __restrict__ u, const int* __restrict__ steps,
                                      float* __restrict__ out, int C, int T, long HW, int tw, int offset) {
    const int b = blockIdx.y;
    const int t0 = steps[b] + offset;
    const long plane = VEC ? HW / 4 : HW;
    const long n = (long)C * tw * plane;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const long p = i % plane;
        const long ct = i / plane;
        const int t = (int)(ct % tw), c = (int)(ct / tw);
        const long src = (((long)b * C + c) * T + t0 + t) * plane + p;
        const long dst = (((long)b * C + c) * tw + t) * plane + p;
        if (VEC)
            reinterpret_cast<f32x4*>(out)[dst] = reinterpret_cast<const f32x4*>(u)[src];
        else
            out[dst] = u[src];
    }
}

}  // namespace

extern "C" int nps_gather_windows(const float* u, const int* steps, float* out, int B, int C, int T, long HW, int tw,
                                  int offset, void* stream) {
    NPS_CHECK_ARG(u && steps && out && B > 0 && C > 0 && T > 0 && HW > 0 && tw > 0, "gather_windows: bad args");
    const bool vec = (HW & 3) == 0 && ((uintptr_t)u & 15) == 0 && ((uintptr_t)out & 15) == 0;
    const long n = (long)C * tw * (vec ? HW / 4 : HW);
    int nb = (int)((n + 255) / 256);
    nb = nb > 4096 ? 4096 : nb;
    if (vec)
        gather_windows_kernel<true><<<dim3(nb, B), 256, 0, (hipStream_t)stream>>>(u, steps, out, C, T, HW, tw, offset);
    else
        gather_windows_kernel<false><<<dim3(nb, B), 256, 0, (hipStream_t)stream>>>(u, steps, out, C, T, HW, tw, offset);
    NPS_CHECK_LAUNCH("gather_windows");
    return 0;
}
