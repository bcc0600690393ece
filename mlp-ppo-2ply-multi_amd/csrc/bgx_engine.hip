// bgx_engine.hip — K4 lane step (select, apply, rewards, records, refill) and
// the 2-ply reductions (K5 top-k / top-5).
//
// One thread per game lane. The lane step restates, per lane:
//   Worker.play_episode (src/multi/worker.py:78-174): pass when no legal
//     move, else V over [obs; candidates], softmax(V[1:]/T) sampling;
//   BackgammonEnv.step (src/environments/backgammon_env.py:130-221): apply,
//     win / gammon / backgammon (2.5 / 2.0 / 1.0), once-per-player close-out
//     (+0.30) and 5-prime (+0.20) shaping summed in fp32, flip, re-roll;
//   BackgammonEnv.reset (backgammon_env.py:92-128): starter roll until not a
//     double (higher first die -> PLAYER1), first roll re-rolled until not a
//     double; episodes end at done or MAX_TIMESTEPS = 300 env steps.
// 2-ply (src/multi/two_ply.py:44-150 + its worker hook 153-193): top-4 by
//   1-ply V, score = alpha*S - beta*sum_rolls P(roll) * mean(top-5 replies),
//   softmax(score/T) over the four; fewer than four moves fall back to 1-ply.
// Dice / sampling randomness: Philox4x32-10 keyed by (seed, global lane id).
#include "bgx_engine.h"

namespace bgx {

__global__ __launch_bounds__(256) void engine_reset_kernel(EngineDev e) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e.L) return;
    LaneRng rng;
    rng.key = lane_key(e.seed, (uint32_t)(e.lane_base + i));
    rng.ctr = 0;
    rng.dt = lane_dice(e, i);
    uint32_t w[8];
    int d0, d1;
    const int p = new_game(rng, w, d0, d1);
    if (rng.exhausted) atomicOr(e.err_flags, BGX_ERRF_DICE_EXHAUSTED);
    store_packed(e.rows + (size_t)i * 8, w);
    e.player[i] = (uint8_t)p;
    e.dice[2 * i] = (uint8_t)d0;
    e.dice[2 * i + 1] = (uint8_t)d1;
    e.step[i] = 0;
    e.flags[i] = 0;
    e.epi[i] = 0;
    e.rng[i] = rng.ctr;
    e.rec_count[i] = 0;
    e.ep_first[i] = 0;
    e.harv[i] = 0;
    if (e.hepi) e.hepi[i] = 0;
}


// Action selection, one wavefront per game lane:
//   1-ply: softmax(V[1:] / T) + Categorical sample (worker.py:137-143);
//   2-ply K=4: score_c = alpha*S_c - beta*W_c for the top-4 (two_ply.py:83-85,
//     W = sum_r P(r) * top-5 mean), softmax(score/T) over the four (two_ply.py
//     hook 153-193); fewer than four moves: 1-ply;
//   2-ply K=all: the same score for every candidate.
// The uniform comes from the lane's Philox stream at its current counter;
// step_lane advances the counter past it. Lane 0 of the wave then runs the
// lane's env step (one launch for select + step).
__global__ __launch_bounds__(256) void select_step_kernel(EngineDev e) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // per-step stats; decisions / episodes are the lanes' own counters
        const unsigned fc = *e.flat_count;
        unsigned long long rows = (unsigned long long)e.L + fc, jobs = (unsigned long long)e.L;
        if (e.ply == 2) {
            rows += *e.reply_count;
            atomicAdd(e.stats + 6, (unsigned long long)*e.reply_count);   // reply rows (gaps included)
            jobs += e.k_top == 0 ? 21ull * fc : (unsigned long long)e.n_jobs2;
        }
        atomicAdd(e.stats + 0, (unsigned long long)e.L);
        atomicAdd(e.stats + 3, rows);
        atomicAdd(e.stats + 4, jobs);
        atomicAdd(e.stats + 5, (unsigned long long)*e.ovf_count + (e.ply == 2 ? *e.ovf_count2 : 0u));
        // last kernel of the step: zero the per-step counters for the next one
        // (no other wave of this kernel reads them)
        *e.flat_count = 0u;
        *e.reply_count = 0u;
        *e.ovf_count = 0u;
        *e.ovf_count2 = 0u;
    }
    // one game lane per half-wave (8 per 256-thread block), as in the fused engine
    __shared__ float xs[8][512];
    const int slot = ((int)threadIdx.x >> 5);
    const int i = blockIdx.x * 8 + slot;
    if (i >= e.L) return;
    const int l = lane_id() & 31;
    const int n_full = e.cand_cnt[i];
    const int n = n_full < e.max_legal ? n_full : e.max_legal;
    if (n == 0) {
        if (l == 0) step_lane(e, i, -1);
        return;
    }
    const int base = e.L + e.cand_off[i];
    const float T = e.temperature;
    const bool k4 = e.ply == 2 && e.k_top == 4 && e.sel[4 * i] >= 0;
    const int m = k4 ? 4 : n;
    float* x = xs[slot];
    for (int k = l; k < m; k += 32) {
        float v;
        if (k4) {
            double W = 0.0;
            const float* jv = e.job_val + (size_t)(4 * i + k) * 21;
            for (int r = 0; r < 21; ++r) W += (double)jv[r] * kRollProbD[r];
            v = (float)((double)e.alpha * (double)e.V[e.sel[4 * i + k]] - (double)e.beta * W) / T;
        } else if (e.ply == 2 && e.k_top == 0) {
            double W = 0.0;
            const float* jv = e.job_val + (size_t)(e.cand_off[i] + k) * 21;
            for (int r = 0; r < 21; ++r) W += (double)jv[r] * kRollProbD[r];
            v = (float)((double)e.alpha * (double)e.V[base + k] - (double)e.beta * W) / T;
        } else {
            v = e.V[base + k] / T;
        }
        x[k] = v;
    }
    wave_sync();
    const int pick = pick_action_half([&](int k) { return x[k]; }, m, e.greedy != 0, lane_uniform(e, i));
    if (l == 0) step_lane(e, i, k4 ? e.sel[4 * i + pick] - base : pick);
}

// 2-ply: top-4 candidates by 1-ply V (torch.topk, sorted; ties -> lower
// index). One wave per lane: each lane keeps the top 4 of its strided
// candidates, then four wave-argmax rounds (value, then lower index) pop the
// overall best.
__global__ __launch_bounds__(256) void topk_kernel(EngineDev e) {
    const int i = blockIdx.x * 4 + ((int)threadIdx.x >> 6);
    if (i >= e.L) return;
    const int l = lane_id();
    const int n_full = e.cand_cnt[i];
    const int n = n_full < e.max_legal ? n_full : e.max_legal;
    const int base = e.L + e.cand_off[i];
    if (n < 4) {
        if (l < 4) {
            e.sel[4 * i + l] = -1;
            uint4* d = (uint4*)(e.sel_rows + (size_t)(4 * i + l) * 8);
            d[0] = make_uint4(0u, 0u, 0u, 0u);
            d[1] = make_uint4(0u, 0u, 0u, 0xFFFFFFFFu);   // SKIP_ROW (bgx_movegen.h)
        }
        return;
    }
    float bv[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int bi[4] = {0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF};
    for (int k = l; k < n; k += 64) {   // ascending k per lane: strict > keeps the lower index first
        const float v = e.V[base + k];
        if (bi[3] != 0x7FFFFFFF && !(v > bv[3])) continue;
        int pos = 3;
        while (pos > 0 && (bi[pos - 1] == 0x7FFFFFFF || v > bv[pos - 1])) {
            bv[pos] = bv[pos - 1];
            bi[pos] = bi[pos - 1];
            --pos;
        }
        bv[pos] = v;
        bi[pos] = k;
    }
    int out = 0;
    for (int c = 0; c < 4; ++c) {
        float v = bv[0];
        int k = bi[0];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const float ov = __shfl_xor(v, off, 64);
            const int ok = __shfl_xor(k, off, 64);
            if (ov > v || (ov == v && ok < k)) { v = ov; k = ok; }
        }
        if (l == c) out = k;
        if (bi[0] == k) {   // the owning lane pops its head
            bv[0] = bv[1]; bv[1] = bv[2]; bv[2] = bv[3]; bv[3] = -INFINITY;
            bi[0] = bi[1]; bi[1] = bi[2]; bi[2] = bi[3]; bi[3] = 0x7FFFFFFF;
        }
    }
    if (l < 4) {
        // the reply launch reads the chosen boards contiguously (no row indirection)
        e.sel[4 * i + l] = base + out;
        const uint4* s = (const uint4*)(e.rows + (size_t)(base + out) * 8);
        uint4* d = (uint4*)(e.sel_rows + (size_t)(4 * i + l) * 8);
        d[0] = s[0];
        d[1] = s[1];
    }
}

// two_ply.py:119-121, reference-sampled mode: a 1-1 / 2-2 / 3-3 job with more
// than sample_k replies keeps a uniformly random sample_k of them
// (random.sample). Reply k is kept iff pi(k) < sample_k, pi a pseudo-random
// permutation of [0, c): a 4-round Feistel network on 10 bits, round keys
// from Philox per (job, step), cycle-walked into [0, c) (c <= 1024; the
// largest reply count seen is 667).
BGX_DEV uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    return x ^ (x >> 16);
}
BGX_DEV uint32_t perm_below(uint32_t x, uint32_t c, const u32x4& key) {
    const uint32_t ks[4] = {key.x, key.y, key.z, key.w};
    do {
        uint32_t L = x >> 5, R = x & 31u;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t t = L ^ (mix32(R ^ ks[r]) & 31u);
            L = R;
            R = t;
        }
        x = (L << 5) | R;
    } while (x >= c);
    return x;
}
BGX_DEV bool small_double(int j) {   // DICE_ROLLS index 0 = 1-1, 6 = 2-2, 11 = 3-3 (two_ply.py:10-32)
    const int r = j % 21;
    return r == 0 || r == 6 || r == 11;
}

// 2-ply: per (candidate, roll) job, mean of the top-5 reply values
// (two_ply.py:133-142); 0 when the opponent has no move (the roll adds nothing).
// A wave takes 16 jobs per iteration, 4 lanes per job: a lane reads the job's
// values k = gl, gl + 4, ... eight loads at a time (issued together) and keeps
// its top 5 with a max / min network; five group-max rounds then pop the
// job's top 5 in descending order (the reference's summation order). The
// lanes of a wave run in lock step, so an iteration costs what its largest job
// costs: the 16 jobs of an iteration are one roll of 16 consecutive
// candidates (jobs (16 b + i) * 21 + r), whose reply counts are alike, not 16
// consecutive rolls of one candidate (a 1-1 with hundreds of replies beside
// fifteen rolls of a dozen). sample_k > 0: the reference-sampled mode above,
// keyed by skey and the step salt *salt_dev (null: 0).
#ifndef BGX_T5_GL
#define BGX_T5_GL 4   // lanes per job (A/B builds: 2, 4, 8)
#endif
#ifndef BGX_T5_VB
#define BGX_T5_VB 0   // > 0: 16-byte block loads, this many per lane per batch (A/B; 0: 8 scalar loads)
#endif
typedef float t5v4 __attribute__((ext_vector_type(4)));
constexpr int T5_GL = BGX_T5_GL;
constexpr int T5_B = 8;    // loads in flight per lane
__global__ __launch_bounds__(256) void top5_kernel(const float* __restrict__ V,
                                                   const int32_t* __restrict__ job_off,
                                                   const int32_t* __restrict__ job_cnt, int n_jobs,
                                                   const unsigned* __restrict__ n_units_dev,
                                                   int jobs_per_unit, int max_jobs, float* __restrict__ out,
                                                   int sample_k, uint64_t skey,
                                                   const unsigned long long* __restrict__ salt_dev,
                                                   unsigned long long* __restrict__ rec_acc) {
    constexpr int JW = 64 / T5_GL;   // jobs per wave iteration
    int nj = n_jobs;
    if (n_units_dev) nj += (int)(*n_units_dev) * jobs_per_unit;
    if (nj > max_jobs) nj = max_jobs;
    const unsigned long long salt = (sample_k > 0 && salt_dev) ? *salt_dev : 0ull;
    const int gl = lane_id() & (T5_GL - 1), q = lane_id() / T5_GL;
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int n_waves = (int)((gridDim.x * blockDim.x) >> 6);
    // iteration it -> (candidate block b, roll r); jobs past nj are inert
    const int n_cand = (nj + 20) / 21;
    const int n_it = ((n_cand + JW - 1) / JW) * 21;
    auto job_of = [&](int it) { return (JW * (it / 21) + q) * 21 + it % 21; };
    int itr = wave;
    int cn = 0, on = 0;
    unsigned long long recs = 0;   // the jobs' records (rec_acc: the engine's reply-record count)
    if (itr < n_it) {
        const int j0 = job_of(itr);
        if (j0 < nj) {
            cn = job_cnt[j0];
            on = job_off[j0];
        }
    }
    for (; itr < n_it; itr += n_waves) {
        const int j = job_of(itr);
        const bool live = j < nj;
        int c = live ? cn : 0;
        const int o = on;
        if (itr + n_waves < n_it) {   // next iteration's job
            const int jn = job_of(itr + n_waves);
            if (jn < nj) {
                cn = job_cnt[jn];
                on = job_off[jn];
            }
        }
        recs += (unsigned long long)c;
        const bool samp = sample_k > 0 && c > sample_k && c <= 1024 && small_double(j);
        u32x4 pk = {0u, 0u, 0u, 0u};
        if (samp) pk = philox(skey, 0x2B1A000000000000ull ^ salt, (uint64_t)j);
        float t[5] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY, -INFINITY};
#if BGX_T5_VB
        // 16-byte blocks: the job's 4 lanes read 64 contiguous bytes per load
        // (one or two cache lines instead of the 8 scalar loads' 8 line
        // accesses per job), blocks aligned on the address: a0 <= o is the
        // first element whose address is 16-byte aligned, so a block may start
        // up to 3 elements before the job and end up to 3 after it; those
        // elements are masked by their index (they belong to other jobs or gap
        // rows, and reading them is in bounds: dalloc pads every buffer by 16 B
        // and a0 >= -3 stays at or after the aligned allocation start)
        // Sampled jobs (rare: 1-1 / 2-2 / 3-3 past sample_k replies) take the
        // scalar loop below: with the permutation's cycle walk inside this
        // loop's unrolled elements, hipcc 7.2 gave wrong, run-dependent top-5s
        // on the GPU (the host emulation of the same source was right).
        const int mis = (int)(((uintptr_t)V >> 2) & 3u);
        const int a0 = ((o + mis) & ~3) - mis, end = samp ? o : o + c;
        for (int b0 = a0 + 4 * gl; b0 < end; b0 += 4 * T5_GL * BGX_T5_VB) {
            t5v4 xb[BGX_T5_VB];
#pragma unroll
            for (int u = 0; u < BGX_T5_VB; ++u) {
                const int i0 = b0 + 4 * T5_GL * u;
                xb[u] = i0 < end ? *(const t5v4*)(V + i0) : t5v4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
            }
#pragma unroll
            for (int u = 0; u < BGX_T5_VB; ++u) {
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                    const int i = b0 + 4 * T5_GL * u + q4;
                    float v = i >= o && i < end ? xb[u][q4] : -INFINITY;
#pragma unroll
                    for (int i5 = 0; i5 < 5; ++i5) {
                        const float hi = fmaxf(t[i5], v);
                        v = fminf(t[i5], v);
                        t[i5] = hi;
                    }
                }
            }
        }
        for (int k0 = gl; samp && k0 < c; k0 += T5_B * T5_GL) {
#else
        for (int k0 = gl; k0 < c; k0 += T5_B * T5_GL) {
#endif
            float xv[T5_B];
#pragma unroll
            for (int u = 0; u < T5_B; ++u) {
                const int k = k0 + T5_GL * u;
                const bool use = k < c && !(samp && perm_below((uint32_t)k, (uint32_t)c, pk) >= (uint32_t)sample_k);
                xv[u] = use ? V[o + k] : -INFINITY;
            }
            // branch-free insert (a max / min network): t stays the lane's top 5
            // in descending order; equal values are interchangeable in the sum
#pragma unroll
            for (int u = 0; u < T5_B; ++u) {
                float v = xv[u];
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    const float hi = fmaxf(t[i], v);
                    v = fminf(t[i], v);
                    t[i] = hi;
                }
            }
        }
        if (samp) c = sample_k;   // the replies kept
        const int m = c < 5 ? c : 5;
        float s = 0.0f;
        for (int r = 0; r < 5; ++r) {
            // the group's largest head (xor-shuffle max over the 4 lanes); the
            // lowest lane holding it pops (ties: lower lane first)
            float mx = t[0];
#pragma unroll
            for (int o = 1; o < T5_GL; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
            const uint32_t grp = (uint32_t)(ballot(t[0] == mx) >> (T5_GL * q)) & ((1u << T5_GL) - 1u);
            const int who = __ffs(grp) - 1;
            if (r < m) s = r ? s + mx : mx;
            if (who == gl) { t[0] = t[1]; t[1] = t[2]; t[2] = t[3]; t[3] = t[4]; t[4] = -INFINITY; }
        }
        if (live && gl == 0) out[j] = m ? s / (float)m : 0.0f;
    }
    if (rec_acc && wave < T5_WAVES) {
        // every lane of a 4-lane group counted its job's c: lanes gl == 0 only.
        // One slot per wave, a plain add (the grid is the same every launch of an
        // engine; a same-address atomic per wave cost ~75 us per launch)
        unsigned long long r = gl == 0 ? recs : 0ull;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) r += __shfl_xor(r, off, 64);
        if (lane_id() == 0 && r) rec_acc[wave] += r;
    }
}

// 2-ply W per board: sum over the 21 rolls of P(roll) * top-5 mean (two_ply.py:143-150)
__global__ __launch_bounds__(256) void two_ply_reduce_kernel(const float* __restrict__ job_val, int n,
                                                             double* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double W = 0.0;
    for (int r = 0; r < 21; ++r) W += (double)job_val[(size_t)i * 21 + r] * kRollProbD[r];
    out[i] = W;
}

// harvest, step 1 (one workgroup): record offsets of the finished episodes
// (exclusive scan of their record counts) and the harvest totals, read on the
// device so the host needs one small copy: info = {episodes, records, error
// flags, episodes appended (incl. any past ep_cap)}; the episode list restarts.
// An episode whose records a lane's ring has already overwritten (harvests
// further apart than the ring allows; flagged BGX_ERRF 8 when it happened) is
// left out: its header's word 15 (0 on the wire) holds its output index, or
// ~0 for a left-out one, for the gather, so the output holds only intact
// episodes and never more records than the rings (L x R).
__global__ __launch_bounds__(1024) void harvest_scan_kernel(EngineDev e, int32_t* __restrict__ offs,
                                                            uint32_t* __restrict__ info, uint32_t* hinfo) {
    __shared__ int wsum[16], wkeep[16];
    const unsigned n_raw = *e.ep_count;
    const int n = (int)n_raw < e.ep_cap ? (int)n_raw : e.ep_cap;
    const int t = (int)threadIdx.x, w = t >> 6;
    int carry = 0, kcarry = 0;
    for (int b = 0; b < n; b += 1024) {
        const int k = b + t;
        int c = 0, keep = 0;
        uint32_t* h = e.ep_list + (size_t)k * EP_WORDS;
        if (k < n) {
            const int lane = (int)h[0] - e.lane_base;
            keep = e.rec_count[lane] - h[2] <= (uint32_t)e.R ? 1 : 0;   // wrap-safe 32-bit distance
            c = keep ? (int)h[3] : 0;
        }
        const int incl = wave_incl_scan(c), kincl = wave_incl_scan(keep);
        if (lane_id() == 63) {
            wsum[w] = incl;
            wkeep[w] = kincl;
        }
        __syncthreads();
        int before = 0, total = 0, kbefore = 0, ktotal = 0;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int x = wsum[q], y = wkeep[q];
            before += q < w ? x : 0;
            total += x;
            kbefore += q < w ? y : 0;
            ktotal += y;
        }
        if (k < n) {
            offs[k] = carry + before + incl - c;
            h[15] = keep ? (uint32_t)(kcarry + kbefore + kincl - 1) : 0xFFFFFFFFu;
        }
        carry += total;
        kcarry += ktotal;
        __syncthreads();
    }
    if (t == 0) {
        offs[n] = carry;
        // the flags of the steps since the previous harvest move into this one's
        // totals (exchanged with 0 in stream order: no host reset of the word
        // while the next step may already run)
        const uint32_t v[4] = {(uint32_t)kcarry, (uint32_t)carry, atomicExch(e.err_flags, 0u), n_raw};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            info[k] = v[k];
            if (hinfo) hinfo[k] = v[k];   // host-mapped (vector stores)
        }
        *e.ep_count = 0u;
    }
    // every finished episode is harvested now (the list holds them all: ep_cap
    // is sized for the steps a ring allows between harvests), so a lane's
    // unharvested records start at its current episode: harv = ep_first (a
    // plain store, wrap-safe for the 32-bit record counters)
    for (int i = t; i < e.L; i += 1024) e.harv[i] = e.ep_first[i];
}

// harvest, step 2: copy finished episodes' headers and records out of the
// lane rings, one wavefront per episode (four per 256-thread block, so 4,096
// episodes are in flight at once), 16 bytes per lane (a record is three
// uint4); persistent grid over the list (info[3], clamped to ep_cap); the
// scan's output index in header word 15 (~0: left out)
__global__ __launch_bounds__(256) void gather_kernel(EngineDev e, const uint32_t* __restrict__ hdr,
                                                     const int32_t* __restrict__ offs,
                                                     const uint32_t* __restrict__ info, uint32_t* __restrict__ hout,
                                                     uint32_t* __restrict__ out) {
    const int n_list = (int)info[3] < e.ep_cap ? (int)info[3] : e.ep_cap;
    constexpr int Q = REC_WORDS / 4;
    const int wpb = (int)blockDim.x >> 6, l = lane_id();
    for (int ep = blockIdx.x * wpb + ((int)threadIdx.x >> 6); ep < n_list; ep += gridDim.x * wpb) {
        const uint32_t* h = hdr + (size_t)ep * EP_WORDS;
        const uint32_t oi = h[15];
        if (oi == 0xFFFFFFFFu) continue;   // its records were overwritten (flagged)
        // the header too: the episode list is refilled by the next step
        if (l < EP_WORDS / 4) {
            uint4 v = ((const uint4*)h)[l];
            if (l == EP_WORDS / 4 - 1) v.w = 0u;   // word 15 is 0 on the wire
            ((uint4*)(hout + (size_t)oi * EP_WORDS))[l] = v;
        }
        const int lane = (int)h[0] - e.lane_base;
        const uint32_t first = h[2], nrec = h[3];
        const uint4* src = (const uint4*)(e.ring + (size_t)lane * e.R * REC_WORDS);
        uint4* dst = (uint4*)(out + (size_t)offs[ep] * REC_WORDS);
        for (uint32_t q = (uint32_t)l; q < nrec * Q; q += 64) {
            const uint32_t r = q / Q, k = q - r * Q;
            const uint32_t slot = (first + r) & (uint32_t)(e.R - 1);
            dst[q] = src[slot * Q + k];
        }
    }
}

// in-kernel harvest (fused engine) with no fused launch since the last ticket:
// the ticket's totals are whatever its commit counter holds (nothing was
// appended); its flags are the accumulator plus any flag raised since (moved,
// not copied)
__global__ void harvest_close_kernel(unsigned long long* commit, unsigned long long* next,
                                     unsigned long long* next_commit, unsigned long long* flags,
                                     unsigned long long* next_flags, unsigned* err_flags, uint32_t* info,
                                     uint32_t* hinfo) {
    const unsigned long long c = *commit;
    const uint32_t fl = atomicExch(err_flags, 0u) | (uint32_t)*flags;
    *flags = fl;
    const uint32_t v[4] = {(uint32_t)(c >> 32), (uint32_t)c, fl, (uint32_t)(c >> 32)};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        info[k] = v[k];
        if (hinfo) hinfo[k] = v[k];
    }
    *next = 0ull;
    *next_commit = 0ull;
    *next_flags = 0ull;
}

}  // namespace bgx

extern "C" hipError_t bgx_launch_harvest_close(unsigned long long* commit, unsigned long long* next,
                                               unsigned long long* next_commit, unsigned long long* flags,
                                               unsigned long long* next_flags, unsigned* err_flags, uint32_t* info,
                                               uint32_t* hinfo, hipStream_t stream) {
    hipLaunchKernelGGL(bgx::harvest_close_kernel, dim3(1), dim3(1), 0, stream, commit, next, next_commit, flags,
                       next_flags, err_flags, info, hinfo);
    return hipGetLastError();
}

extern "C" hipError_t bgx_launch_engine_reset(const bgx::EngineDev* e, hipStream_t stream) {
    hipLaunchKernelGGL(bgx::engine_reset_kernel, dim3((e->L + 255) / 256), dim3(256), 0, stream, *e);
    return hipGetLastError();
}

extern "C" hipError_t bgx_launch_select(const bgx::EngineDev* e, hipStream_t stream) {
    hipLaunchKernelGGL(bgx::select_step_kernel, dim3((e->L + 7) / 8), dim3(256), 0, stream, *e);
    return hipGetLastError();
}
extern "C" hipError_t bgx_launch_topk(const bgx::EngineDev* e, hipStream_t stream) {
    hipLaunchKernelGGL(bgx::topk_kernel, dim3((e->L + 3) / 4), dim3(256), 0, stream, *e);
    return hipGetLastError();
}
extern "C" hipError_t bgx_launch_top5(const float* V, const int32_t* job_off, const int32_t* job_cnt,
                                      int n_jobs, const unsigned* n_units_dev, int jobs_per_unit,
                                      int max_jobs, float* out, int sample_k, uint64_t skey,
                                      const unsigned long long* salt_dev, unsigned long long* rec_acc,
                                      hipStream_t stream) {
    if (max_jobs <= 0) return hipSuccess;
    constexpr int jw = 64 / bgx::T5_GL;                 // jobs per wave iteration, 4 waves per block
    int blocks = (max_jobs + 4 * jw - 1) / (4 * jw);
    if (blocks > bgx::T5_WAVES / 4) blocks = bgx::T5_WAVES / 4;   // 8 waves per SIMD on 256 CUs, then loop
    hipLaunchKernelGGL(bgx::top5_kernel, dim3(blocks), dim3(256), 0, stream, V, job_off, job_cnt, n_jobs,
                       n_units_dev, jobs_per_unit, max_jobs, out, sample_k, skey, salt_dev, rec_acc);
    return hipGetLastError();
}
extern "C" hipError_t bgx_launch_two_ply_reduce(const float* job_val, int n, double* out,
                                                 hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(bgx::two_ply_reduce_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, job_val, n,
                       out);
    return hipGetLastError();
}
extern "C" hipError_t bgx_launch_harvest_scan(const bgx::EngineDev* e, int32_t* offsets, uint32_t* info,
                                              uint32_t* hinfo, hipStream_t stream) {
    hipLaunchKernelGGL(bgx::harvest_scan_kernel, dim3(1), dim3(1024), 0, stream, *e, offsets, info, hinfo);
    return hipGetLastError();
}

extern "C" hipError_t bgx_launch_harvest_gather(const bgx::EngineDev* e, const int32_t* offsets, const uint32_t* info,
                                                uint32_t* hout, uint32_t* out, hipStream_t stream) {
    hipLaunchKernelGGL(bgx::gather_kernel, dim3(1024), dim3(256), 0, stream, *e, e->ep_list, offsets, info, hout,
                       out);
    return hipGetLastError();
}
