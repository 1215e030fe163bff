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
    printf("calibration: full 1 GiB, half 0.5 GiB, halves 0.5 + 0.5 GiB (dispatches 1, 2, 3+4)\n");
    hipFree(x);
    hipFree(sink);
    return 0;
}
