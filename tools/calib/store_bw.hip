// Store-throughput calibration for the conv epilogues (dev tool, not product).  One 512-thread work-group
// per CU walks 96-KiB output tiles of a 1.5 GiB NHWC buffer (192 channels x 4 B per pixel, 128 pixels per
// tile) the way the conv epilogues store them, optionally interleaved with a read stream, and reports the
// chip-wide rate.  Shapes:
//   coal   : 16 B per lane, consecutive lanes consecutive (x3_store_phase)
//   frag   : the MFMA accumulator layout (store_tile): lane (pixel l & 31, half h) writes 16 B at channel
//            8m + 4h of 32-channel block cb, 24 instructions per wave for 32 pixels x 192 channels
//   *_rd   : the same plus a read of 2 x the tile's bytes per tile (a 1x1's input stream), loads first
// Each variant: 3 warm-up launches, then 10 timed with hipEvents.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool FRAG, bool RD>
__global__ __launch_bounds__(512) void store_kernel(f32x4* __restrict__ out, const f32x4* __restrict__ in, long ntiles,
                                                    float* sink) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    f32x4 s = {1.f, 2.f, 3.f, 4.f};
    for (long t = blockIdx.x; t < ntiles; t += gridDim.x) {
        if (RD) {  // 192 KiB of reads per tile: 24 x 16 B per thread, issued together
            const f32x4* src = in + t * 12288;
            f32x4 r[24];
#pragma unroll
            for (int i = 0; i < 24; ++i) r[i] = src[i * 512 + tid];
#pragma unroll
            for (int i = 0; i < 24; ++i) s += r[i];
        }
        f32x4* dst = out + t * 6144;  // 96 KiB = 6144 f32x4
        if (!FRAG) {
#pragma unroll
            for (int i = 0; i < 12; ++i) dst[i * 512 + tid] = s;
        } else if (wave < 4) {  // 4 MFMA waves x 32 pixels x 192 channels (48 f32x4 per pixel)
            const int px = wave * 32 + (lane & 31), h = lane >> 5;
#pragma unroll
            for (int cb = 0; cb < 6; ++cb)
#pragma unroll
                for (int m = 0; m < 4; ++m) dst[px * 48 + cb * 8 + 2 * m + h] = s;
        }
    }
    if (s[0] == 12345.f) sink[0] = 1.f;
}

template <bool FRAG, bool RD>
void run(const char* name, f32x4* out, const f32x4* in, long ntiles, float* sink, int grid) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) store_kernel<FRAG, RD><<<grid, 512>>>(out, in, ntiles, sink);
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) store_kernel<FRAG, RD><<<grid, 512>>>(out, in, ntiles, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 10.f;
    const double wb = ntiles * 98304.0, rb = RD ? ntiles * 196608.0 : 0.0;
    printf("%-8s grid %4d: %.3f ms  write %.2f TB/s  read %.2f TB/s  total %.2f TB/s  (%.0f cycles per tile per CU at 2 GHz)\n",
           name, grid, ms, wb / ms / 1e9, rb / ms / 1e9, (wb + rb) / ms / 1e9, ms * 1e-3 * 2e9 / ((double)ntiles / grid));
}

int main() {
    const long ntiles = 16384;  // 1.5 GiB of output
    f32x4 *out, *in;
    float* sink;
    if (hipMalloc(&out, ntiles * 98304) != hipSuccess || hipMalloc(&in, ntiles * 196608) != hipSuccess ||
        hipMalloc(&sink, 64) != hipSuccess)
        return 1;
    hipMemset(in, 0, ntiles * 196608);
    int ncu = 256;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    for (int grid : {32, 64, 128, ncu}) {
        run<false, false>("coal", out, in, ntiles, sink, grid);
        run<true, false>("frag", out, in, ntiles, sink, grid);
        run<false, true>("coal_rd", out, in, ntiles, sink, grid);
        run<true, true>("frag_rd", out, in, ntiles, sink, grid);
    }
    hipFree(out);
    hipFree(in);
    hipFree(sink);
    return 0;
}
