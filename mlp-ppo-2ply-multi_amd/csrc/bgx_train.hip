// bgx_train.hip — the TD(0) consumer on the device: the
// reference's per-episode update loop (src/agents/trainer.py:81-138) as ONE
// launch over a harvest's episodes, instead of a dozen eager torch launches and
// a host sync per episode (bgx/trainer.py's torch path, kept as the checker).
//
// Per episode, in order (each episode starts from the previous one's weights):
//   Y = V(observations)            (trainer.py:106-107; x = the live 198-feature
//                                   encoding of the record's board + mover flag)
//   target = rewards, + gamma * Y[1:] (detached) on all but the last step (110-114)
//   loss = mean((Y - target)^2)    (117)
//   grads by backprop              (120-121)
//   clip_grad_norm_(params, clip)  (124-127: coef = clip / (norm + 1e-6), <= 1)
//   Adam (lr, betas (0.9, 0.999), eps 1e-8, torch's update order) (138)
//
// One 512-thread workgroup. Thread (j, q) = (tid >> 2, tid & 3) owns hidden
// unit j's W1 columns [52q, 52q + 52) (198 real) and their gradient
// accumulators, in registers for the whole launch (the Adam moments are read
// and written in place once per episode); the 4 threads of a
// unit are adjacent lanes (their partial dot products combine by two xor
// shuffles in a fixed order). Thread t < 257 also owns small parameter t (b1,
// then w2, then b2). LDS holds a chunk of 64 observations (fp32 features), the
// chunk's sigmoid activations (then their backprop terms) and the episode's V
// values. fp32 throughout; the summation orders differ from torch's GEMMs
// (last-bit differences), the per-episode sequence and the optimizer
// arithmetic follow torch's.
#include "bgx_device.h"
#include "bgx_kernels.h"

namespace bgx {

constexpr int TR_T = 512;                 // threads (two waves per SIMD: 256 registers)
constexpr int TR_Q = 4, TR_W = 52;        // threads per hidden unit, W1 columns per thread (198 = 3 x 52 + 42)
constexpr int TR_TC = 64;                 // observations per chunk
constexpr int TR_KP = 208;                // padded feature stride (198 + 10 zeros; 16-byte slices)
constexpr int N_W1 = 128 * 198, N_SMALL = 128 + 128 + 1;

// feature f of the live encoding (immutable_board.py:86-128) of packed words w[0..6]
BGX_DEV float live_feature(const uint32_t* w, int f) {
    if (f >= 198) return 0.0f;
    const uint32_t s6 = w[6];
    if (f >= 196) return (int)((s6 >> 16) & 1u) == f - 196 ? 1.0f : 0.0f;
    if (f >= 192) {
        const int k = f - 192, who = k >> 1;   // bar1, off1, bar2, off2
        const uint32_t v = (s6 >> (4 * who + ((k & 1) ? 8 : 0))) & 15u;
        return (k & 1) ? (float)((double)v / 15.0) : (float)v * 0.5f;
    }
    const int pl = f / 96, rest = f - 96 * pl, i = rest >> 2;
    const int n = (int)((w[3 * pl + (i >> 3)] >> ((i & 7) * 4)) & 15u);
    switch (rest & 3) {
        case 0: return n >= 1 ? 1.0f : 0.0f;
        case 1: return n >= 2 ? 1.0f : 0.0f;
        case 2: return n >= 3 ? 1.0f : 0.0f;
        default: return n > 3 ? (float)(n - 3) * 0.5f : 0.0f;
    }
}

BGX_DEV float sum4(float v) {   // the 4 adjacent lanes of a hidden unit, fixed order
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    return v;
}

// Workgroup barrier for LDS only: the kernel's global memory is either read
// only (records) or owned by one thread (weights, moments), so a barrier need
// not drain the Adam moments' stores (__syncthreads' release fence would).
BGX_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int N>
BGX_DEV void block_sums(float* v, float* red) {   // N sums over all threads, the same results everywhere
    const int t = (int)threadIdx.x;
#pragma unroll
    for (int k = 0; k < N; ++k)
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v[k] += __shfl_xor(v[k], off, 64);
    lds_barrier();
    if ((t & 63) == 0)
#pragma unroll
        for (int k = 0; k < N; ++k) red[k * (TR_T / 64) + (t >> 6)] = v[k];
    lds_barrier();
#pragma unroll
    for (int k = 0; k < N; ++k) {
        float s = 0.0f;
#pragma unroll
        for (int w = 0; w < TR_T / 64; ++w) s += red[k * (TR_T / 64) + w];
        v[k] = s;
    }
}

#ifdef BGX_TRAIN_STAMP
static __device__ unsigned long long bgx_train_stamps[16];
#define TSTAMP(k)                                                                   \
    do {                                                                            \
        const unsigned long long c_ = __builtin_amdgcn_s_memtime();               \
        if (threadIdx.x == 0) { tsum[k] += c_ - tlast; }                           \
        tlast = c_;                                                                 \
    } while (0)
#else
#define TSTAMP(k)
#endif

__global__ __launch_bounds__(TR_T) void td0_train_kernel(TrainArgs a) {
#ifdef BGX_TRAIN_STAMP
    unsigned long long tsum[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tlast = __builtin_amdgcn_s_memtime();
#endif
    __shared__ __attribute__((aligned(16))) float X[TR_TC][TR_KP];   // observations of the chunk
    __shared__ float S[TR_TC][128];           // sigmoid(h), then dL/dh
    __shared__ float Y[TRAIN_TMAX];           // V of the episode's observations
    __shared__ float DY[TR_TC];               // dL/dV of the chunk
    __shared__ uint32_t RW[TR_TC][7];         // the chunk's record boards
    __shared__ float red[4 * TR_T / 64];
    __shared__ float sps[N_SMALL];            // b1 | w2 | b2 of the current weights
    const int t = (int)threadIdx.x, j = t / TR_Q, q = t % TR_Q, k0 = TR_W * q;
    const int kn = q == TR_Q - 1 ? 198 - TR_W * (TR_Q - 1) : TR_W;

    // ---- weights into registers (the Adam moments stay in global memory /
    // L2 and are read and written once per episode, in the update)
    float W[TR_W], G[TR_W];
    const int pbase = j * 198 + k0;           // the thread's first W1 entry (flat)
#pragma unroll
    for (int i = 0; i < TR_W; ++i) W[i] = i < kn ? a.params[pbase + i] : 0.0f;
    const bool small = t < N_SMALL;
    float sp = small ? a.params[N_W1 + t] : 0.0f;
    float sm = small ? a.adam_m[N_W1 + t] : 0.0f;
    float sv = small ? a.adam_v[N_W1 + t] : 0.0f;
    int step = *a.step;
    double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};   // thread 0: loss, post-clip norm, |td| mean, V mean, reward

    for (int e = 0; e < a.n_eps; ++e) {
        const int r0 = a.offs[e], T = a.offs[e + 1] - r0;
        if (T <= 0 || T > TRAIN_TMAX) continue;   // (the host validates)
        if (small) sps[t] = sp;
        lds_barrier();
        const float* b1s = sps;
        const float* w2s = sps + 128;
        const float bias2 = sps[256];
        float gS = 0.0f;                           // small parameter t's gradient
#pragma unroll
        for (int i = 0; i < TR_W; ++i) G[i] = 0.0f;

        auto load_chunk = [&](int c0, int n) {    // X[0..n) = features of records r0 + c0 ..
            // the chunk's records (words 0..6: the board before the move, the
            // mover's flag) into LDS with one coalesced pass, then the features
            for (int idx = t; idx < n * 7; idx += TR_T) {
                const int r = idx / 7, k = idx - 7 * r;
                RW[r][k] = a.rec[(size_t)(r0 + c0 + r) * 12 + k];
            }
            lds_barrier();
            for (int idx = t; idx < n * TR_KP; idx += TR_T) {
                const int r = idx / TR_KP, f = idx - r * TR_KP;
                X[r][f] = live_feature(RW[r], f);
            }
            lds_barrier();
        };
        auto forward_chunk = [&](int c0, int n) {  // S = sigmoid(W1 x + b1); Y[c0 + r] = w2 . S + b2
#pragma unroll 1
            for (int r = 0; r < n; ++r) {
                float p = 0.0f;
                const float4* xr = (const float4*)&X[r][k0];
#pragma unroll
                for (int i4 = 0; i4 < TR_W / 4; ++i4) {
                    const float4 x = xr[i4];
                    p = fmaf(W[4 * i4], x.x, p);
                    p = fmaf(W[4 * i4 + 1], x.y, p);
                    p = fmaf(W[4 * i4 + 2], x.z, p);
                    p = fmaf(W[4 * i4 + 3], x.w, p);
                }
                const float h = sum4(p) + b1s[j];
                if (q == 0) S[r][j] = 1.0f / (1.0f + expf(-h));
            }
            lds_barrier();
            if (t < n) {
                float y = 0.0f;
                for (int u = 0; u < 128; ++u) y = fmaf(w2s[u], S[t][u], y);
                Y[c0 + t] = y + bias2;
            }
            lds_barrier();
        };

        TSTAMP(0);
        // ---- pass 1: V of every observation (the targets need V[s + 1])
        for (int c0 = 0; c0 < T; c0 += TR_TC) {
            const int n = T - c0 < TR_TC ? T - c0 : TR_TC;
            load_chunk(c0, n);
            TSTAMP(1);
            forward_chunk(c0, n);
            TSTAMP(2);
        }
        // ---- pass 2: backprop, chunk by chunk from the last (still in LDS)
        float loss_p = 0.0f, td_p = 0.0f, y_p = 0.0f, rw_p = 0.0f;
        const int last0 = ((T - 1) / TR_TC) * TR_TC;
        for (int c0 = last0; c0 >= 0; c0 -= TR_TC) {
            const int n = T - c0 < TR_TC ? T - c0 : TR_TC;
            if (c0 != last0) {
                load_chunk(c0, n);
                forward_chunk(c0, n);
            }
            if (t < n) {
                const int s = c0 + t;
                const float rew = __uint_as_float(a.rec[(size_t)(r0 + s) * 12 + 9]);
                const float tg = s + 1 < T ? rew + a.gamma * Y[s + 1] : rew;
                const float d = Y[s] - tg;
                DY[t] = 2.0f * d / (float)T;   // d mean((y - tg)^2) / dy
                loss_p += d * d;
                td_p += fabsf(tg - Y[s]);
                y_p += Y[s];
                rw_p += rew;
            }
            lds_barrier();
            // w2 / b2 gradients from the activations: dw2_u = sum_r dy_r s_ru, db2 = sum_r dy_r
            if (t >= 128 && t < 256) {
                for (int r = 0; r < n; ++r) gS = fmaf(DY[r], S[r][t - 128], gS);
            } else if (t == 256) {
                for (int r = 0; r < n; ++r) gS += DY[r];
            }
            lds_barrier();
            // dL/dh = ((dy w2) (1 - s)) s  (torch's sigmoid_backward order)
            for (int idx = t; idx < n * 128; idx += TR_T) {
                const int r = idx >> 7, u = idx & 127;
                const float s = S[r][u];
                S[r][u] = ((DY[r] * w2s[u]) * (1.0f - s)) * s;
            }
            lds_barrier();
            // dW1[j][k] += dh_rj x_rk; db1_j += dh_rj
#pragma unroll 1
            for (int r = 0; r < n; ++r) {
                const float gh = S[r][j];
                const float4* xr = (const float4*)&X[r][k0];
#pragma unroll
                for (int i4 = 0; i4 < TR_W / 4; ++i4) {
                    const float4 x = xr[i4];
                    G[4 * i4] = fmaf(gh, x.x, G[4 * i4]);
                    G[4 * i4 + 1] = fmaf(gh, x.y, G[4 * i4 + 1]);
                    G[4 * i4 + 2] = fmaf(gh, x.z, G[4 * i4 + 2]);
                    G[4 * i4 + 3] = fmaf(gh, x.w, G[4 * i4 + 3]);
                }
            }
            if (t < 128)
                for (int r = 0; r < n; ++r) gS += S[r][t];
            lds_barrier();
        }
        TSTAMP(3);
        // ---- clip_grad_norm_ (trainer.py:124-127)
        float sq = small ? gS * gS : 0.0f;
#pragma unroll
        for (int i = 0; i < TR_W; ++i) sq = fmaf(G[i], G[i], sq);
        block_sums<1>(&sq, red);
        const float norm = sqrtf(sq);
        float scale = 1.0f;
        if (a.grad_clip > 0.0f) {
            const float coef = a.grad_clip / (norm + 1e-6f);
            scale = coef < 1.0f ? coef : 1.0f;
#pragma unroll
            for (int i = 0; i < TR_W; ++i) G[i] *= scale;
            gS *= scale;
        }
        // ---- Adam (torch.optim.Adam, non-capturable: bias corrections in double)
        ++step;
        const double bc1 = 1.0 - pow(0.9, (double)step), bc2 = 1.0 - pow(0.999, (double)step);
        const float step_size = (float)(a.lr / bc1);
        const float w1m = (float)(1.0 - 0.9), w2v = (float)(1.0 - 0.999);
        // the update is the whole CU's work per episode (25,729 parameters), so
        // its square root and division are the hardware's (v_sqrt / v_rcp,
        // ~1 ulp) instead of the correctly rounded sequences
        const float inv_bc2s = (float)(1.0 / sqrt(bc2));
        auto adam = [&](float& p, float& m, float& v, float g) {
            m = m + w1m * (g - m);                 // lerp(m, g, 1 - beta1)
            v = v * 0.999f + w2v * g * g;          // mul(beta2).addcmul(g, g, 1 - beta2)
            const float den = __builtin_amdgcn_sqrtf(v) * inv_bc2s + 1e-8f;   // sqrt(v) / sqrt(bc2) + eps
            p = p + (-step_size) * (m * __builtin_amdgcn_rcpf(den));          // addcdiv(m, den, -step_size)
        };
        {
            // moments four at a time, the next four loaded before this group's
            // stores are issued (vmcnt counts loads and stores in issue order:
            // a load behind a store would wait for the store's acknowledgement)
            // (uniform base + 32-bit per-lane offset: the SGPR-based addressing)
            float* __restrict__ gm = a.adam_m;
            float* __restrict__ gv = a.adam_v;
            constexpr int NG = TR_W / 4;
            float mb[2][4], vb[2][4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                mb[0][u] = u < kn ? gm[pbase + u] : 0.0f;
                vb[0][u] = u < kn ? gv[pbase + u] : 0.0f;
            }
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                const int cur = g & 1, nxt = cur ^ 1;
                if (g + 1 < NG) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int i = 4 * (g + 1) + u;
                        mb[nxt][u] = i < kn ? gm[pbase + i] : 0.0f;
                        vb[nxt][u] = i < kn ? gv[pbase + i] : 0.0f;
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int i = 4 * g + u;
                    if (i < kn) {
                        adam(W[i], mb[cur][u], vb[cur][u], G[i]);
                        gm[pbase + i] = mb[cur][u];
                        gv[pbase + i] = vb[cur][u];
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (small) adam(sp, sm, sv, gS);
        TSTAMP(4);
        // ---- metrics (DeviceTrainer's: loss, post-clip norm, |td| mean, V mean, reward sum)
        float sums[4] = {loss_p, td_p, y_p, rw_p};
        block_sums<4>(sums, red);
        const float ls = sums[0], tds = sums[1], ys = sums[2], rws = sums[3];
        if (t == 0) {
            acc[0] += (double)(ls / (float)T);
            acc[1] += (double)(norm * scale);
            acc[2] += (double)(tds / (float)T);
            acc[3] += (double)(ys / (float)T);
            acc[4] += (double)rws;
        }
        lds_barrier();
        TSTAMP(5);
    }
#ifdef BGX_TRAIN_STAMP
    if (threadIdx.x == 0)
        for (int k = 0; k < 6; ++k) bgx_train_stamps[k] += tsum[k];
#endif
    // ---- state back
#pragma unroll
    for (int i = 0; i < TR_W; ++i)
        if (i < kn) a.params[pbase + i] = W[i];
    if (small) {
        a.params[N_W1 + t] = sp;
        a.adam_m[N_W1 + t] = sm;
        a.adam_v[N_W1 + t] = sv;
    }
    if (t == 0) {
        *a.step = step;
        for (int k = 0; k < 5; ++k) a.metrics[k] += acc[k];
    }
}

}  // namespace bgx

#ifdef BGX_TRAIN_STAMP
extern "C" int bgx_diag_train_stamps(unsigned long long* out6) {
    return hipMemcpyFromSymbol(out6, HIP_SYMBOL(bgx::bgx_train_stamps), 6 * 8) == hipSuccess ? 0 : -1;
}
#endif

extern "C" hipError_t bgx_launch_td0(const bgx::TrainArgs* args, hipStream_t stream) {
    if (args->n_eps <= 0) return hipSuccess;
    hipLaunchKernelGGL(bgx::td0_train_kernel, dim3(1), dim3(bgx::TR_T), 0, stream, *args);
    return hipGetLastError();
}
