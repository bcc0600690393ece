// tests/cpuwave/hip/hip_runtime.h -- test infrastructure, NOT product code.
// A host emulation of one 64-lane wavefront for the movegen device headers
// (csrc/bgx_movegen.h, bgx_device.h): each lane is a host thread, every
// cross-lane operation (ballot, shuffles, readlane, DPP) is an exchange
// through a shared buffer between two barriers, so code whose cross-lane
// operations are reached by every lane runs as on the GPU, and host tools
// (AddressSanitizer) see its LDS slices and output buffers. Only what those
// headers use is provided.
#pragma once
#include <algorithm>
#include <atomic>
#include <barrier>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <type_traits>
#include <memory>
#include <vector>

#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __launch_bounds__(...)
typedef int hipError_t;
typedef void* hipStream_t;

struct alignas(16) uint4 { uint32_t x, y, z, w; };
inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return {x, y, z, w}; }
struct emu_dim3 { unsigned x, y, z; };
struct alignas(16) float4 { float x, y, z, w; };
struct float2 { float x, y; };

namespace emu {
// one emulated wavefront: its exchange buffer and its 64-lane barrier
struct Wave {
    std::barrier<>* bar = nullptr;
    alignas(16) unsigned char xbuf[64][64];
};
inline thread_local int lane = 0;          // lane in the wave
inline thread_local int tid = 0;           // thread in the workgroup
inline thread_local unsigned block = 0;    // workgroup index
inline thread_local Wave* cur = nullptr;   // this thread's wave (null: the single wave below)
inline unsigned grid = 1, block_threads = 64;
inline std::barrier<>* bar = nullptr;      // single-wave programs (dbl_check): its barrier
inline Wave single;
inline std::barrier<>* block_bar = nullptr;
inline Wave& W() {
    if (cur) return *cur;
    single.bar = bar;
    return single;
}
#ifdef EMU_TRACE
}  // namespace emu
#include <execinfo.h>
namespace emu {
inline void* where[1024][8];
inline int nwhere[1024];
inline unsigned long long nsync[1024];
inline void sync() {
    nwhere[tid] = backtrace(where[tid], 8);
    ++nsync[tid];
    W().bar->arrive_and_wait();
}
#else
inline void sync() { W().bar->arrive_and_wait(); }
#endif
// EMU_SITES: every exchange also checks that the 64 lanes reached it from the
// same call site (build with -O0 -fno-inline so sites stay distinct): a
// cross-lane operation under lane-divergent control flow reads inactive lanes
// on the GPU, which this emulation would otherwise hide
#ifdef EMU_SITES
inline void* site_buf[32][64][8];
inline int site_n[32][64];
}  // namespace emu
#include <cstdio>
#include <execinfo.h>
namespace emu {
#endif
// every lane's v (as 64-bit words)
template <class T> __attribute__((noinline)) inline void gather(T v, T* out) {
    static_assert(sizeof(T) <= 64, "exchange of at most 64 bytes per lane");
    Wave& w = W();
    std::memcpy(w.xbuf[lane], &v, sizeof(T));
#ifdef EMU_SITES
    const int widx = cur ? tid >> 6 : 0;
    site_n[widx][lane] = backtrace(site_buf[widx][lane], 8);   // the whole call chain (up to 8 frames)
#endif
    sync();
#ifdef EMU_SITES
    if (lane == 0)
        for (int i = 1; i < 64; ++i)
            if (site_n[widx][i] != site_n[widx][0] ||
                std::memcmp(site_buf[widx][i], site_buf[widx][0], sizeof(void*) * site_n[widx][0])) {
                fprintf(stderr, "EMU_SITES: lanes 0 and %d of wave %d exchange at different call chains:\n", i, widx);
                for (int k = 0; k < 8; ++k)
                    fprintf(stderr, "  %p %p\n", k < site_n[widx][0] ? site_buf[widx][0][k] : nullptr,
                            k < site_n[widx][i] ? site_buf[widx][i][k] : nullptr);
                std::abort();
            }
#endif
    for (int i = 0; i < 64; ++i) std::memcpy(&out[i], w.xbuf[i], sizeof(T));
    sync();
}
template <class T> inline T lane_value(T v, int k) {
    T all[64];
    gather(v, all);
    return all[k & 63];
}
}  // namespace emu

#define threadIdx (emu_dim3{(unsigned)(emu::cur ? emu::tid : emu::lane), 0u, 0u})
#define blockIdx (emu_dim3{emu::block, 0u, 0u})
#define gridDim (emu_dim3{emu::grid, 1u, 1u})
#define blockDim (emu_dim3{emu::block_threads, 1u, 1u})

inline unsigned __lane_id() { return (unsigned)emu::lane; }
inline uint64_t __ballot(bool p) {
    bool all[64];
    emu::gather(p, all);
    uint64_t m = 0;
    for (int i = 0; i < 64; ++i) m |= (uint64_t)all[i] << i;
    return m;
}
template <class T> inline T __shfl(T v, int src, int width = 64) { (void)width; return emu::lane_value(v, src); }
template <class T> inline T __shfl_xor(T v, int m, int width = 64) { (void)width; return emu::lane_value(v, emu::lane ^ m); }
inline int __popc(uint32_t v) { return __builtin_popcount(v); }
inline int __popcll(uint64_t v) { return __builtin_popcountll(v); }
inline int __ffs(uint32_t v) { return __builtin_ffs((int)v); }
inline int __ffsll(uint64_t v) { return __builtin_ffsll((long long)v); }
inline int __clz(uint32_t v) { return v ? __builtin_clz(v) : 32; }
inline int __clzll(long long v) { return v ? __builtin_clzll((unsigned long long)v) : 64; }
inline uint32_t __umulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
inline float __int_as_float(int v) { float f; std::memcpy(&f, &v, 4); return f; }
inline int __float_as_int(float f) { int v; std::memcpy(&v, &f, 4); return v; }
inline unsigned long long wall_clock64() { return 0ull; }
inline void __syncthreads() {
    if (emu::block_bar) emu::block_bar->arrive_and_wait();
    else emu::sync();
}

#define __builtin_amdgcn_readlane(v, k) emu::lane_value((int)(v), (int)(k))
#define __builtin_amdgcn_readfirstlane(v) emu::lane_value((int)(v), 0)
#define __builtin_amdgcn_s_memtime() 0ull
#define __builtin_amdgcn_s_sleep(n) std::this_thread::yield()
#define __builtin_amdgcn_fence(...) std::atomic_thread_fence(std::memory_order_seq_cst)
#define __builtin_amdgcn_wave_barrier() emu::sync()
inline uint32_t emu_mbcnt_lo(uint32_t m, uint32_t acc) {
    const int l = emu::lane;
    return acc + (uint32_t)__builtin_popcount(l >= 32 ? m : (m & ((1u << l) - 1u)));
}
inline uint32_t emu_mbcnt_hi(uint32_t m, uint32_t acc) {
    const int l = emu::lane;
    return acc + (uint32_t)(l < 32 ? 0 : __builtin_popcount(m & (uint32_t)((1ull << (l - 32)) - 1ull)));
}
#define __builtin_amdgcn_mbcnt_lo(m, acc) emu_mbcnt_lo((m), (acc))
#define __builtin_amdgcn_mbcnt_hi(m, acc) emu_mbcnt_hi((m), (acc))
// DPP for the controls the headers use: row_shr:1..15 (0x111..0x11F),
// row_bcast:15 (0x142), row_bcast:31 (0x143)
inline int emu_update_dpp(int old, int src, int ctrl, int row_mask, int bank_mask, bool bound_ctrl) {
    (void)bank_mask;
    int all[64];
    emu::gather(src, all);
    const int l = emu::lane, row = l >> 4;
    if (!((row_mask >> row) & 1)) return old;
    int from = -1;
    if (ctrl >= 0x111 && ctrl <= 0x11F) {
        const int n = ctrl - 0x110;
        if ((l & 15) >= n) from = l - n;
    } else if (ctrl == 0x142) {
        if (row >= 1) from = 16 * row - 1;
    } else if (ctrl == 0x143) {
        if (row >= 2) from = 31;
    } else {
        std::abort();
    }
    if (from < 0) return bound_ctrl ? 0 : old;
    return all[from];
}
#define __builtin_amdgcn_update_dpp(old, src, ctrl, rm, bm, bc) emu_update_dpp((old), (src), (ctrl), (rm), (bm), (bc))

#define __HIP_MEMORY_SCOPE_WAVEFRONT 1
#define __HIP_MEMORY_SCOPE_WORKGROUP 2
#define __HIP_MEMORY_SCOPE_AGENT 3
#define __HIP_MEMORY_SCOPE_SYSTEM 4
#define __hip_atomic_load(p, order, scope) __atomic_load_n((p), __ATOMIC_SEQ_CST)
#define __hip_atomic_store(p, v, order, scope) __atomic_store_n((p), (v), __ATOMIC_SEQ_CST)
template <class T> inline T emu_fetch_min(T* p, std::type_identity_t<T> v) {
    T cur = __atomic_load_n(p, __ATOMIC_SEQ_CST);
    while (v < cur && !__atomic_compare_exchange_n(p, &cur, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
    }
    return cur;
}
#define __hip_atomic_fetch_min(p, v, order, scope) emu_fetch_min((p), (v))
#define __hip_atomic_fetch_add(p, v, order, scope) __atomic_fetch_add((p), (v), __ATOMIC_SEQ_CST)
#define __hip_atomic_compare_exchange_strong(p, cmp, v, o1, o2, scope) \
    __atomic_compare_exchange_n((p), (cmp), (v), false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)
template <class T> inline T atomicAdd(T* p, std::type_identity_t<T> v) { return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST); }
template <class T> inline T atomicOr(T* p, std::type_identity_t<T> v) { return __atomic_fetch_or(p, v, __ATOMIC_SEQ_CST); }
template <class T> inline T atomicMin(T* p, std::type_identity_t<T> v) { return emu_fetch_min(p, v); }
template <class T> inline T atomicCAS(T* p, std::type_identity_t<T> cmp, std::type_identity_t<T> v) {
    __atomic_compare_exchange_n(p, &cmp, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
    return cmp;
}

// ---- workgroup launches (movegen launchers compiled for the host): every
// workgroup of the grid in turn, its threads as host threads, one 64-lane
// barrier per wave and one workgroup barrier; __shared__ variables become
// function statics (the workgroups run one after another)
#define __shared__ static
struct dim3 {
    unsigned x, y, z;
    dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};
#define hipSuccess 0
#define hipDeviceAttributeMultiprocessorCount 0
inline int emu_n_cu = 2;
inline hipError_t hipGetLastError() { return hipSuccess; }
inline hipError_t hipGetDevice(int* d) { *d = 0; return hipSuccess; }
// EMU_N_CU: the emulated compute units (grid sizes of the persistent launchers; default 2)
inline hipError_t hipDeviceGetAttribute(int* v, int attr, int dev) {
    (void)attr;
    (void)dev;
    const char* e = getenv("EMU_N_CU");
    *v = e ? atoi(e) : emu_n_cu;
    return hipSuccess;
}
template <class F> inline hipError_t hipOccupancyMaxActiveBlocksPerMultiprocessor(int* n, F, int, size_t) {
    *n = 1;
    return hipSuccess;
}
inline hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t) { std::memset(p, v, n); return hipSuccess; }
namespace emu {
inline void* dyn_lds = nullptr;   // the workgroup's dynamic LDS (extern __shared__ arrays)
template <class K, class... A> inline void launch(K kernel, unsigned g, unsigned nthreads, size_t shmem, A... args) {
    const unsigned nw = nthreads / 64;
    std::vector<unsigned long long> dyn((shmem + 7) / 8 + 1);
    dyn_lds = dyn.data();
    grid = g;
    block_threads = nthreads;
    for (unsigned b = 0; b < g; ++b) {
        std::vector<Wave> waves(nw);
        std::vector<std::unique_ptr<std::barrier<>>> bars;
        for (unsigned w = 0; w < nw; ++w) {
            bars.emplace_back(new std::barrier<>(64));
            waves[w].bar = bars.back().get();
        }
        std::barrier<> bb((std::ptrdiff_t)nthreads);
        block_bar = &bb;
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nthreads; ++t)
            th.emplace_back([&, t] {
                tid = (int)t;
                lane = (int)(t & 63u);
                block = b;
                cur = &waves[t >> 6];
                kernel(args...);
                // a thread that returns early must keep its wave's and the
                // workgroup's barriers moving for the others
                cur->bar->arrive_and_drop();
                block_bar->arrive_and_drop();
            });
        for (auto& x : th) x.join();
        block_bar = nullptr;
    }
    dyn_lds = nullptr;
}
}  // namespace emu
#define hipLaunchKernelGGL(kernel, g, b, shmem, stream, ...) \
    emu::launch(kernel, dim3(g).x, dim3(b).x, (size_t)(shmem), __VA_ARGS__)

// ---- MLP kernels: math builtins, LDS-DMA, MFMA (clang host builds: ext_vector_type, _Float16)
#define __builtin_amdgcn_exp2f(x) std::exp2((float)(x))
#define __builtin_amdgcn_rcpf(x) (1.0f / (float)(x))
#define __builtin_amdgcn_sched_barrier(n) ((void)0)
#define __builtin_amdgcn_s_waitcnt(n) ((void)0)
#define __builtin_amdgcn_s_setprio(n) ((void)0)
// global -> LDS, size bytes per lane: lane l's bytes land at the (wave-uniform)
// LDS address + l * size
#define __builtin_amdgcn_global_load_lds(g, l, size, off, aux) \
    std::memcpy((char*)(void*)(l) + (size_t)emu::lane * (size), (const void*)(g), (size))
// v_mfma_f32_32x32x16_f16: D[i][j] = C[i][j] + sum_k A[i][k] B[k][j] (i, j < 32, k < 16);
// lane l holds A[l % 32][8 (l / 32) + e] and B[8 (l / 32) + e][l % 32] (e < 8), and
// D[8 (r / 4) + 4 (l / 32) + r % 4][l % 32] in accumulator register r
template <class HA, class HB, class FC> inline FC emu_mfma_32x32x16(HA a, HB b, FC c) {
    HA A[64];
    HB B[64];
    emu::gather(a, A);
    emu::gather(b, B);
    const int l = emu::lane, j = l & 31;
    FC d;
    for (int r = 0; r < 16; ++r) {
        const int i = 8 * (r >> 2) + 4 * (l >> 5) + (r & 3);
        float acc = 0.0f;
        for (int k = 0; k < 16; ++k) acc += (float)A[i + 32 * (k >> 3)][k & 7] * (float)B[j + 32 * (k >> 3)][k & 7];
        d[r] = c[r] + acc;
    }
    return d;
}
#define __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, x, y, z) emu_mfma_32x32x16((a), (b), (c))
#define hipFuncAttributeMaxDynamicSharedMemorySize 0
#define hipErrorInvalidValue 1
template <class F> inline hipError_t hipFuncSetAttribute(F, int, int) { return hipSuccess; }
