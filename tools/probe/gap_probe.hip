// Launch-gap probe (tools only): back-to-back dependent kernels on one stream
// with different block shapes / LDS sizes; run under rocprofv3 --kernel-trace
// and compare start(k+1) - end(k).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_small(int* p) { if (threadIdx.x == 0) atomicAdd(p, 1); }
__global__ __launch_bounds__(1024) void k_big_static(int* p) {
    __shared__ int s[110 * 1024 / 4];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(p, s[5]);
}
__global__ __launch_bounds__(512) void k_big_dyn(int* p) {
    extern __shared__ int s[];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(p, s[7]);
}
__global__ __launch_bounds__(64) void k_wave8k(int* p) {
    __shared__ int s[2048];
    s[threadIdx.x] = threadIdx.x;
    if (threadIdx.x == 0) atomicAdd(p, s[3]);
}

int main() {
    int* d;
    hipMalloc(&d, 4);
    hipFuncSetAttribute((const void*)k_big_dyn, hipFuncAttributeMaxDynamicSharedMemorySize, 108 * 1024);
    hipStream_t s;
    hipStreamCreate(&s);
    for (int it = 0; it < 200; ++it) {
        hipLaunchKernelGGL(k_wave8k, dim3(5120), dim3(64), 0, s, d);      // tier-1 shape
        hipLaunchKernelGGL(k_big_static, dim3(256), dim3(1024), 0, s, d);  // tier-2 shape
        hipLaunchKernelGGL(k_big_dyn, dim3(256), dim3(512), 108 * 1024, s, d);  // mlp shape
        hipLaunchKernelGGL(k_small, dim3(64), dim3(64), 0, s, d);          // select shape
        hipLaunchKernelGGL(k_small, dim3(64), dim3(64), 0, s, d);          // step shape
    }
    hipStreamSynchronize(s);
    printf("done\n");
    return 0;
}
