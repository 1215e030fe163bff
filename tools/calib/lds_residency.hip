// Residency calibration (dev tool): how many 256-thread work-groups per CU gfx950 admits at a given
// dynamic LDS size.  Each work-group touches its LDS, holds ~20 us, and records s_memrealtime at start /
// end; the host prints the peak number resident at once for each LDS size.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void hold_kernel(unsigned long long* t, int lds_floats) {
    extern __shared__ float s[];
    for (int i = threadIdx.x; i < lds_floats; i += 256) s[i] = (float)i;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(10);  // 20 us at 100 MHz
    if (threadIdx.x == 0) {
        t[2 * blockIdx.x] = t0;
        t[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
    if (s[threadIdx.x] < -1.f) t[0] = 0;  // keep the LDS live
}

int main() {
    const int nwg = 4096;
    unsigned long long* d;
    if (hipMalloc(&d, sizeof(unsigned long long) * 2 * nwg) != hipSuccess) return 1;
    (void)hipFuncSetAttribute((const void*)hold_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    std::vector<unsigned long long> h(2 * nwg);
    for (int kb : {16, 24, 32, 40, 48, 53, 56, 64, 80, 96}) {
        hold_kernel<<<nwg, 256, kb * 1024>>>(d, kb * 256);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        if (hipMemcpy(h.data(), d, sizeof(unsigned long long) * 2 * nwg, hipMemcpyDeviceToHost) != hipSuccess) return 3;
        std::vector<std::pair<unsigned long long, int>> ev;
        for (int i = 0; i < nwg; ++i) {
            ev.push_back({h[2 * i], +1});
            ev.push_back({h[2 * i + 1], -1});
        }
        std::sort(ev.begin(), ev.end());
        int cur = 0, peak = 0;
        for (auto& e : ev) peak = std::max(peak, cur += e.second);
        printf("dynamic LDS %3d KiB: peak resident work-groups %d (%.2f per CU of 256)\n", kb, peak, peak / 256.0);
    }
    (void)hipFree(d);
    return 0;
}
