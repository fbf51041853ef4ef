// Write-bandwidth probe (r04): how fast can a pure store stream go on this MI355X?  The
// conv_first_fwd pass writes 545 MB (config 2) and reads almost nothing; this measures plain
// vs nontemporal dwordx4 stores of the same size, grid-stride and block-contiguous, and a
// float4 copy for reference.  hipcc --offload-arch=gfx950 -O3 tools/wbw.hip -o tools/bin/wbw
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void store_k(f4* __restrict__ y, long n4, int per) {
    if (MODE == 2) {  // block-contiguous ranges, U = 4 stores in flight per trip
        const long b0 = (long)blockIdx.x * per;
        const long b1 = b0 + per < n4 ? b0 + per : n4;
        for (long i = b0 + threadIdx.x; i < b1; i += 1024) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u * 256 < b1) y[i + u * 256] = f4{1.f, 2.f, 3.f, (float)u};
        }
        return;
    }
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        const f4 v = {1.f, 2.f, 3.f, (float)(i & 7)};
        if (MODE == 1)
            __builtin_nontemporal_store(v, y + i);
        else
            y[i] = v;
    }
}

__global__ __launch_bounds__(256) void copy_k(const f4* __restrict__ x, f4* __restrict__ y, long n4) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) y[i] = x[i];
}

int main() {
    const long bytes = 545259520L;  // 32 x 256 x 256 x 64 floats
    const long n4 = bytes / 16;
    f4 *x, *y;
    if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&y, bytes) != hipSuccess) return 1;
    hipMemset(x, 0, bytes);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int grid : {2048, 8192, 32768}) {
        for (int mode = 0; mode < 4; ++mode) {
            const int per = (int)((n4 + grid - 1) / grid);
            float best = 1e9f;
            for (int r = 0; r < 6; ++r) {
                hipEventRecord(a);
                if (mode == 0) hipLaunchKernelGGL(store_k<0>, dim3(grid), dim3(256), 0, 0, y, n4, per);
                if (mode == 1) hipLaunchKernelGGL(store_k<1>, dim3(grid), dim3(256), 0, 0, y, n4, per);
                if (mode == 2) hipLaunchKernelGGL(store_k<2>, dim3(grid), dim3(256), 0, 0, y, n4, per);
                if (mode == 3) hipLaunchKernelGGL(copy_k, dim3(grid), dim3(256), 0, 0, x, y, n4);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                if (r > 0 && ms < best) best = ms;
            }
            const double moved = mode == 3 ? 2.0 * bytes : (double)bytes;
            printf("grid %6d mode %d (%s): %.3f ms  %.2f TB/s\n", grid, mode,
                   mode == 0 ? "store" : mode == 1 ? "nt store" : mode == 2 ? "block-range x4" : "copy",
                   best, moved / best / 1e9);
        }
    }
    return 0;
}
