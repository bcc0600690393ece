// Dispatch probe (tools only): 5120 trivial waves launched as blocks of
// 64 / 256 / 512 / 1024 threads, with and without 8 KB of LDS per wave; run
// under rocprofv3 --kernel-trace and compare kernel durations.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int T, int LDS_PER_WAVE>
__global__ __launch_bounds__(T) void k_trivial(int* p) {
    if constexpr (LDS_PER_WAVE > 0) {
        __shared__ int s[(T / 64) * LDS_PER_WAVE / 4];
        s[threadIdx.x] = threadIdx.x;
        __syncthreads();
        if (threadIdx.x == 0 && s[3] == 12345) atomicAdd(p, 1);
    } else {
        if (threadIdx.x == 0 && p[1] == 12345) atomicAdd(p, 1);
    }
}

template <int T, int L>
void run(hipStream_t s, int* d) {
    hipLaunchKernelGGL((k_trivial<T, L>), dim3(5120 * 64 / T), dim3(T), 0, s, d);
}

int main() {
    int* d;
    (void)hipMalloc(&d, 8);
    (void)hipMemset(d, 0, 8);
    hipStream_t s;
    (void)hipStreamCreate(&s);
    for (int it = 0; it < 50; ++it) {
        run<64, 0>(s, d);
        run<64, 8192>(s, d);
        run<256, 0>(s, d);
        run<256, 8192>(s, d);
        run<512, 0>(s, d);
        run<512, 8192>(s, d);
        run<1024, 0>(s, d);
        run<1024, 8192>(s, d);
    }
    (void)hipStreamSynchronize(s);
    printf("done\n");
    return 0;
}
