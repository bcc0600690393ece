// bgx_kernels.h — launch-argument structs shared by the kernels and the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bgx.h"   // BGX_BADF_* (input-domain bits)

#define BGX_ERRF_FLAT_OVERFLOW 1u       // flat reply buffer too small
#define BGX_ERRF_OVF_LIST 2u            // overflow job list too small
#define BGX_ERRF_FALLBACK_OVERFLOW 4u   // a job outgrew the global workspace
#define BGX_ERRF_RING_OVERFLOW 8u       // experience ring overwritten before harvest
#define BGX_ERRF_EPISODE_LIST 16u       // finished-episode list full
#define BGX_ERRF_DICE_EXHAUSTED 32u     // a lane read past its scripted dice (bgx_engine_set_dice)
#define BGX_ERRF_WAIT_BOUND 64u         // an intra-workgroup wait hit its iteration bound (reported as BGX_E_STATE)

namespace bgx {

enum InMode { IN_U8 = 0, IN_PACKED = 1, IN_TWOPLY = 2 };
enum OutMode { OUT_U8 = 0, OUT_PACKED_SLOT = 1, OUT_PACKED_FLAT = 2 };

struct MovegenArgs {
    int n_jobs;                  // host job count (added to the device count below)
    const unsigned* n_jobs_dev;  // optional: device count of "units"
    int jobs_per_dev_unit;       //   ... each giving this many jobs (21 for 2-ply rows)
    int n_jobs_max;              // > 0: clamp the job count (capacity of the per-job arrays)
    int in_mode;
    const uint8_t* in_u8;        // IN_U8: [n][52]
    const uint32_t* in_packed;   // IN_PACKED: [n][8]; IN_TWOPLY: candidate rows [*][8]
    const uint8_t* in_player;    // [n]
    const uint8_t* in_dice;      // [n][2]
    const int32_t* in_rows;      // IN_TWOPLY: [n/21] candidate row (or -1 = skip);
    int in_row_base;             //   if in_rows == nullptr: row = in_row_base + job / 21
    int out_mode;
    int cap;                     // per-job output capacity (U8 / SLOT)
    uint8_t* out_u8;             // [n][cap][52]
    uint32_t* out_packed;        // SLOT: [n][cap][8]; FLAT: [flat_cap][8]
    int32_t* out_count;          // [n] full record count (U8 / SLOT)
    unsigned* flat_count;        // FLAT: running row count
    int flat_cap;
    int flat_chunk;              // FLAT: rows a wave reserves per global atomic (0 = exact per job;
                                 //   > 0 leaves unused gap rows that downstream kernels tolerate)
    int32_t* job_off;            // FLAT: [n]
    int32_t* job_cnt;            // FLAT: [n]
    // overflow handling (doubles whose frontier outgrows the LDS slice)
    unsigned* ovf_count;
    int32_t* ovf_list;
    int ovf_cap;
    uint32_t* ws_global;         // [ws_waves][ws_words_per_wave]
    int ws_waves;
    int ws_slots;                // power of two
    size_t ws_words_per_wave;    // >= 5 * ws_slots
    int ovf_zeroed;              // caller zeroed *ovf_count on the stream already (skip the memset)
    int heavy_t;                 // set by the launcher: doubles level size handed to the block tier
    int force_table;             // test hook (BGX_MG_TEST_TABLE=1): every job takes the hash-table path
                                 //   (no table-free doubles / non-doubles rules), as a cross-check
    int force_tier;              // test hook (BGX_MG_TEST_TIER): 2/3 = skip the LDS tiers below
    int reply_groups;            // tools hook (BGX_REPLY_GROUPS, tools/reply_micro.py): run only the
                                 //   reply items of these groups (bit 0: non-doubles, bit d: (d, d)); 0 = all;
                                 //   0x80: leave roots board_nd_records does not cover out; 0x100: treat
                                 //   every root as not covered
    int dbl_tail64;              // set by the launcher (board-major doubles reply launch): the last
                                 //   dbl_tail64 / 64 of the rows run one item per doubles roll
    unsigned* err_flags;
};

// Split-fp16 MLP weights in MFMA fragment order (see bgx_mlp.hip).
struct MlpArgs {
    const uint32_t* rows;        // packed boards [n][8] (flag in w[6] bit 16)
    const unsigned* n_rows_dev;  // if non-null: row count read on device
    int n_rows;                  // else: row count
    int n_max;                   // capacity of rows/out: the device count is clamped to it
    int nt;                      // 32-board tiles per wave iteration: 1 (small batches) or 2
    float* out;                  // [n] V
    const uint4* wfrag;          // [2][4][13][64] fragments (16 B each)
    const float* rowc;           // [128] w2 (value_head.weight)
    float b2;
    float feat_scale;            // 2^-e: features are scaled so the accumulator is -h log2(e)
    // nt = 1 kernel (the 2-ply root launch): rows >= z_base also write their 128
    // hidden-layer accumulators to zout[row - z_base][2][4][16] (lane half h,
    // m-tile, accumulator register: the order mlp_kernel_delta reads them in)
    float* zout;
    int z_base;
    // the 2-ply reply launch by difference (mlp_kernel_delta, when zt is set):
    // row word 7 = its root slot; root row = root_sel ? root_sel[slot] :
    // root_base + slot, clamped to [root_base, root_base + n_roots); its packed
    // board at root_rows[root row], its accumulators at zt[root row - root_base]
    const float* zt;
    const uint32_t* root_rows;
    const int32_t* root_sel;
    int root_base;
    int n_roots;
    int n_slots;                 // root slots (clamp of word 7)
};

// Self-play lane state (one engine per device), structure of arrays.
// Experience record (48 B; include/bgx.h bgx_harvest): words 0..6 the packed
// board before the move (word 6 bit 16 = the mover), 7 V(s), 8 V(a), 9 reward,
// 10 action | n_moves << 11 | step << 23, 11 dice0 | dice1 << 3 | done << 6 |
// close_out << 7 | prime << 8 | mover << 9 | win_type << 10. The board after
// the move is the next record's before-board (passes do not move checkers), or
// for an episode's last record the final board in its header.
constexpr int REC_WORDS = 12;
// Episode header (64 B): global lane, episode no., first record, n_records,
// env steps, win_type | winner << 8 | flags << 16, final board words 0..6, 0, 0, 0
constexpr int EP_WORDS = 16;

struct EngineDev {
    int L;                       // lanes on this engine
    int lane_base;               // global id of lane 0 (RNG streams keyed by global id)
    uint64_t seed;
    float temperature;
    int max_steps;               // MAX_TIMESTEPS = 300 (config/configuration.py:4)
    int max_legal;               // max_legal_moves = 500 (backgammon_env.py:35)
    int ply;                     // 1 or 2
    int k_top;                   // 4 (two_ply.py:67-70) or 0 = all candidates
    float alpha, beta;           // 1.0, 0.9 (two_ply.py:44-50)
    int greedy;                  // argmax instead of sampling (play_versus_ai.py:188-195)
    uint32_t* rows;              // [L + cand_cap][8]: lane boards (obs rows) then candidates
    int cand_cap;
    uint8_t* player;             // [L]
    uint8_t* dice;               // [L][2]
    int32_t* step;               // [L] env steps in the current episode (passes included)
    uint32_t* flags;             // [L] bit0/1 close-out given P1/P2, bit2/3 prime given, bit4/5 decided
    uint32_t* epi;               // [L] episode counter
    uint64_t* rng;               // [L] Philox counter
    uint32_t* rec_count;         // [L] records written (absolute)
    uint32_t* ep_first;          // [L] first record of the current episode
    uint32_t* harv;              // [L] records harvested (absolute)
    uint32_t* ring;              // [L][R][REC_WORDS]
    int R;                       // ring slots per lane (a power of two: slot = record counter & (R - 1))
    const uint8_t* dice_tab;     // test hook (bgx_engine_set_dice): [L][dice_len] scripted single-die draws, or null
    int dice_len;
    uint32_t* ep_list;           // [ep_cap][EP_WORDS]
    unsigned* ep_count;
    int ep_cap;
    // fused engine: finished-episode headers go to a per-lane ring instead of
    // ep_list, so a fused workgroup harvests its own lanes at the end of a
    // launch (FusedArgs hv_*); null on the phased engines
    uint32_t* hring;             // [L][HR][EP_WORDS], slot = episode number & (HR - 1)
    int HR;                      // header slots per lane (a power of two)
    uint32_t* hepi;              // [L] episodes harvested (absolute episode number)
    // per-step inputs
    const int32_t* cand_off;     // [L] offset of the lane's candidates after row L
    const int32_t* cand_cnt;     // [L] full candidate count
    const float* V;              // [L + cand rows] values
    int32_t* sel;                // [L * 4] 2-ply: candidate rows chosen by 1-ply V (or -1)
    uint32_t* sel_rows;          // [L * 4][8] 2-ply: those rows' packed boards (word 7 = SKIP_ROW: none)
    const float* job_val;        // [L * 4 * 21] 2-ply: top-5 mean per (candidate, roll)
    unsigned* flat_count;        // candidate rows this step (device; zeroed by the step kernel)
    unsigned* reply_count;       // 2-ply reply rows this step (device; zeroed by the step kernel)
    unsigned* ovf_count;         // jobs sent to the fallback path this step (device)
    unsigned* ovf_count2;        // same, for the 2-ply reply launch
    int n_jobs2;                 // 2-ply jobs this step when k_top = 4
    unsigned long long* stats;   // [8] env steps, decisions, episodes, value rows, movegen jobs, fallback
    unsigned* err_flags;
};

// Fused 1-ply lane step (bgx_fused.hip): one persistent launch runs n_steps
// env steps of every lane; the 16 or 32 lanes of a workgroup advance together.
struct FusedArgs {
    EngineDev e;
    uint32_t* cand;              // [L][cap][8] packed candidate rows, lane-major
    float* vbuf;                 // [L][cap + 1] V(s), then V(candidate k) at 1 + k
    int cap;                     // candidate slots per lane (= max_legal: later moves are never read)
    int n_steps;
    const uint4* wfrag;          // split-fp16 W fragments (MlpArgs::wfrag)
    const float* rowc;           // [128] w2
    float b2;
    float feat_scale;
    uint32_t* ws_global;         // tier-3 movegen workspace, one slice per workgroup
    int ws_blocks;               // slices (>= gridDim.x)
    int ws_slots;
    size_t ws_words_per_block;
    int force_tier;              // test hook (BGX_MG_TEST_TIER)
    unsigned long long* prof;    // development (BGX_FUSED_PROF): [gridDim.x][16] phase clocks, or null
    int lanes_per_wg;            // 16 or 32 game lanes per workgroup; 0: the launcher picks (32 when
                                 //   every CU still gets a workgroup)
    // balanced launch (bgx_config.balance): each workgroup-step takes a ticket of
    // its lanes from budget_ctr[0] and steps while the running total is below
    // `budget` lane-steps, at most n_cap steps; budget <= 0: every lane runs
    // exactly n_steps (lockstep). The last workgroup to finish (done_ctr) zeroes
    // budget_ctr (zero at engine create) for the next launch. The launcher
    // balances only when each workgroup owns one lane group.
    long long budget;
    int n_cap;
    unsigned long long* budget_ctr;
    // the next step's tier-1 results carried between launches: the last step
    // of a launch also expands its lanes' next positions (into `cand`) and
    // stores each lane's count (-1: tier 2) in t1cnt[lane]; t1_ready = the
    // previous launch did so and nothing changed the lanes since (the host
    // clears it on every reset), so the next launch starts at tier 2
    int* t1cnt;
    int t1_ready;
    // in-kernel harvest (fused engine): each workgroup, once its lanes are done
    // for the launch, appends their finished episodes (headers from e.hring,
    // records from the lane rings) to this ticket's output at offsets from one
    // 64-bit atomic (episodes << 32 | records) and sets the lanes' harvested
    // marks; the last workgroup to finish moves the engine's error flags into
    // this output's accumulator (atomic exchange with 0, so the flags of the
    // launches since the previous ticket belong to this ticket alone), publishes
    // the totals {episodes, records, error flags, episodes} to hv_info /
    // hv_hinfo and zeroes the next output's counter and flags. hv_hdr null: no
    // harvest in this launch.
    uint32_t* hv_hdr;            // [ep cap][EP_WORDS]
    uint32_t* hv_rec;            // [L * R][REC_WORDS]
    int hv_ep_cap;               // headers the output holds
    long long hv_rec_cap;        // records the output holds (L x R)
    unsigned long long* hv_ctr;  // this output's reservations (fetch-add of a group's totals)
    unsigned long long* hv_next; // the next output's (zeroed by the last workgroup)
    unsigned long long* hv_commit;       // this output's totals: the groups that fit (published)
    unsigned long long* hv_next_commit;  // the next output's (zeroed by the last workgroup)
    unsigned long long* hv_flags;       // this output's accumulated error flags
    unsigned long long* hv_next_flags;  // the next output's (zeroed by the last workgroup)
    uint32_t* hv_info;           // [4] device
    uint32_t* hv_hinfo;          // [4] host-mapped
    unsigned long long* done_ctr;   // finished workgroups of the launch (the last one zeroes it)
};

// TD(0) trainer (bgx_train.hip): one launch over n_eps episodes of compact
// records (12 words each; the episode e is records [offs[e], offs[e + 1])).
constexpr int TRAIN_TMAX = 2048;   // longest episode (records) the trainer accepts
struct TrainArgs {
    const uint32_t* rec;         // [m][12] experience records (bgx/records.py layout)
    const int32_t* offs;         // [n_eps + 1]
    int n_eps;
    float* params;               // fc1.weight [128][198] | fc1.bias [128] | value_head.weight [128] | value_head.bias
    float* adam_m;               // Adam first / second moments, same layout
    float* adam_v;
    int* step;                   // Adam step count
    float lr, gamma, grad_clip;  // grad_clip <= 0: no clipping
    double* metrics;             // [5] += loss, post-clip grad norm, |td| mean, V mean, reward sum (per episode)
};

// the 2-ply top-5 launch: at most this many waves (2,048 blocks of 4), each
// with its own record-count slot (bgx_launch_top5's rec_acc)
constexpr int T5_WAVES = 2048 * 4;

}  // namespace bgx

extern "C" {
hipError_t bgx_launch_movegen(const bgx::MovegenArgs* args, hipStream_t stream);
hipError_t bgx_launch_mlp(const bgx::MlpArgs* args, hipStream_t stream);
hipError_t bgx_launch_fused(const bgx::FusedArgs* args, hipStream_t stream);
// input-domain check (flags[0] = BGX_BADF_* bits, flags[1] = first bad index)
hipError_t bgx_launch_validate(const uint8_t* boards, const uint8_t* player, const uint8_t* dice, int n,
                               unsigned* flags, hipStream_t stream);
hipError_t bgx_launch_encode(const uint8_t* boards, const uint8_t* player, int n, float* out,
                             int layout, hipStream_t stream);
hipError_t bgx_launch_encode_packed(const uint32_t* packed, int n, float* out, int layout, hipStream_t stream);
hipError_t bgx_launch_value_f32(const float* x, int n, const float* W1, const float* b1,
                                const float* w2, float b2, float* out, hipStream_t stream);
hipError_t bgx_launch_pack(const uint8_t* boards, const uint8_t* player, int n, uint32_t* out,
                           hipStream_t stream);
hipError_t bgx_launch_unpack(const uint32_t* packed, int n, uint8_t* out, hipStream_t stream);
hipError_t bgx_launch_engine_reset(const bgx::EngineDev* e, hipStream_t stream);
hipError_t bgx_launch_topk(const bgx::EngineDev* e, hipStream_t stream);
hipError_t bgx_launch_select(const bgx::EngineDev* e, hipStream_t stream);   // select + env step
hipError_t bgx_launch_top5(const float* V, const int32_t* job_off, const int32_t* job_cnt, int n_jobs,
                           const unsigned* n_units_dev, int jobs_per_unit, int max_jobs, float* out,
                           int sample_k, uint64_t skey, const unsigned long long* salt_dev,
                           unsigned long long* rec_acc, hipStream_t stream);   // rec_acc[wave] += its jobs' records
                                                                     // (bgx::T5_WAVES slots, or null)
hipError_t bgx_launch_two_ply_reduce(const float* job_val, int n, double* out, hipStream_t stream);
hipError_t bgx_launch_td0(const bgx::TrainArgs* args, hipStream_t stream);
// harvest: episode offsets / totals (info[4] on the device, hinfo[4] host-mapped
// or null), then the headers + records gather (persistent grid; the episode
// count is read on the device)
hipError_t bgx_launch_harvest_scan(const bgx::EngineDev* e, int32_t* offsets, uint32_t* info, uint32_t* hinfo,
                                   hipStream_t stream);
// in-kernel harvest bookkeeping when no fused launch ran since the last ticket:
// publish the (empty) totals of ctr with the accumulated error flags (the
// engine's flags moved in) and zero the next output's counter and flags
hipError_t bgx_launch_harvest_close(unsigned long long* commit, unsigned long long* next, unsigned long long* next_commit,
                                    unsigned long long* flags, unsigned long long* next_flags, unsigned* err_flags,
                                    uint32_t* info, uint32_t* hinfo, hipStream_t stream);
hipError_t bgx_launch_harvest_gather(const bgx::EngineDev* e, const int32_t* offsets, const uint32_t* info,
                                     uint32_t* hout, uint32_t* out, hipStream_t stream);
}
