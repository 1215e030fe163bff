// FETCH_SIZE calibration for the access shapes of the split-fp16 conv producers (dev tool, not product).
// MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of the bytes of a wide coalesced (16 B/lane) streaming read;
// other shapes are uncalibrated.  The conv producers read 64 B (16 channels x 4 B) of each pixel per stage,
// the other 64 B of the 128-B line one stage later.  Three kernels over a 1 GiB buffer (4x the Infinity
// Cache), each launched alone so rocprofv3 --pmc FETCH_SIZE reports it per dispatch:
//   full   : 16 B per lane, consecutive lanes consecutive (every byte once)             -> 1 GiB
//   half   : lane quads read the first 64 B of each 128-B line (pixel pitch 128 B)      -> 0.5 GiB
//   halves : the same, then (after the whole sweep) the second 64 B of every line       -> 1 GiB
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void full_kernel(const f32x4* __restrict__ x, long n4, float* sink) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) s += x[i];
    if (s[0] + s[1] + s[2] + s[3] == 12345.f) sink[0] = 1.f;
}

// line l = 128 B = 8 f32x4; lane quad q reads f32x4 (8 l + 4 half + q)
__global__ void half_kernel(const f32x4* __restrict__ x, long lines, int half, float* sink) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    const long nq = lines * 4;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nq; i += (long)gridDim.x * blockDim.x)
        s += x[(i >> 2) * 8 + half * 4 + (i & 3)];
    if (s[0] + s[1] + s[2] + s[3] == 12345.f) sink[0] = 1.f;
}

// LDS-DMA full-line sweep (the 1x1 DMA kernel's input shape): global_load_lds_dwordx4, 16 B per lane,
// 8 lanes per 128-B line, every byte once
__global__ void dma_kernel(const f32x4* __restrict__ x, long n4) {
    __shared__ __attribute__((aligned(16))) f32x4 buf[256];
    const int wave = threadIdx.x >> 6;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const unsigned*>(x + i),
                                         (__attribute__((address_space(3))) unsigned*)(buf + wave * 64), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// the register-staged 1x1's B-operand shape (conv1x1_wl_kernel): per instruction, lane (pixel l & 31, half
// h = l >> 5) reads 16 B at byte 64 h + 16 q of its pixel's 128-B stage line; q = 0..3 in 4 instructions
__global__ void pair_kernel(const f32x4* __restrict__ x, long lines, float* sink) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    const int lane = threadIdx.x & 63;
    const long nw = (long)gridDim.x * (blockDim.x >> 6);
    for (long g = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); g * 32 < lines; g += nw) {
        const long l = g * 32 + (lane & 31);
        if (l >= lines) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) s += x[l * 8 + (lane >> 5) * 4 + q];
    }
    if (s[0] + s[1] + s[2] + s[3] == 12345.f) sink[0] = 1.f;
}
// stores, WRITE_SIZE: coalesced 16 B per lane (x3_store_phase), and the MFMA accumulator fragment shape
// (store_tile / the 1x1 epilogues: per instruction 32 pixels x 32 B at a 768-B pixel pitch), every byte once
__global__ void store_coal_kernel(f32x4* __restrict__ x, long n4) {
    const f32x4 v = {1.f, 2.f, 3.f, 4.f};
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) x[i] = v;
}
__global__ void store_frag_kernel(f32x4* __restrict__ x, long npx) {  // npx pixels of 48 f32x4, 32 per wave
    const f32x4 v = {1.f, 2.f, 3.f, 4.f};
    const int lane = threadIdx.x & 63;
    const long nw = (long)gridDim.x * (blockDim.x >> 6);
    for (long g = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); g * 32 < npx; g += nw) {
        const long px = g * 32 + (lane & 31);
        const int h = lane >> 5;
        if (px >= npx) continue;
#pragma unroll
        for (int cb = 0; cb < 6; ++cb)
#pragma unroll
            for (int m = 0; m < 4; ++m) x[px * 48 + cb * 8 + 2 * m + h] = v;
    }
}

int main() {
    const size_t bytes = 1ull << 30;
    f32x4* x;
    float* sink;
    if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
    hipMemset(x, 0, bytes);
    hipDeviceSynchronize();
    const long n4 = bytes / 16, lines = bytes / 128;
    const dim3 g(2048), b(256);
    full_kernel<<<g, b>>>(x, n4, sink);
    hipDeviceSynchronize();
    half_kernel<<<g, b>>>(x, lines, 0, sink);
    hipDeviceSynchronize();
    half_kernel<<<g, b>>>(x, lines, 0, sink);   // "halves": first halves ...
    half_kernel<<<g, b>>>(x, lines, 1, sink);   // ... then second halves
    hipDeviceSynchronize();
    dma_kernel<<<g, b>>>(x, n4);
    hipDeviceSynchronize();
    pair_kernel<<<g, b>>>(x, lines, sink);
    hipDeviceSynchronize();
    store_coal_kernel<<<g, b>>>(x, n4);
    hipDeviceSynchronize();
    store_frag_kernel<<<g, b>>>(x, (long)(bytes / 768));
    hipDeviceSynchronize();
    printf("calibration: full 1 GiB, half 0.5 GiB, halves 0.5 + 0.5 GiB (dispatches 1, 2, 3+4); dma 1 GiB read (5); "
           "pair 1 GiB read (6); store_coal 1 GiB written (7), store_frag 1 GiB written (8)\n");
    hipFree(x);
    hipFree(sink);
    return 0;
}
