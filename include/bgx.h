/*
 * bgx.h — C-ABI of libbgx.so, the MI355X (gfx950) self-play engine for the
 * backgammon TD learner of Nick-qsv/MLP-PPO-2PLY-MULTI.
 *
 * The reference has no native boundary; its hot path is Python called in
 * process by the rollout worker. Each entry point below states the reference
 * interface it replaces (file:line under the reference's src/). A Python
 * ctypes binding that mirrors the reference's src/multi surface is shipped in
 * mlp-ppo-2ply-multi_amd/bgx; INTEGRATION.md shows the stub a maintainer adds.
 *
 * Conventions
 *  - Every call returns int: 0 = ok, < 0 = error (BGX_E_*); the message of
 *    the last error on the calling thread is bgx_last_error(). No exceptions,
 *    aborts or printing cross the ABI.
 *  - Pointers named d_* are DEVICE pointers (e.g. torch .data_ptr() of a
 *    cuda tensor) and calls taking `stream` (a hipStream_t, NULL = default)
 *    are asynchronous on it. Pointers named h_* are host pointers.
 *  - Boards are the reference's ImmutableBoard fields as u8[52]:
 *    positions_0[24] | positions_1[24] | bar[2] | borne_off[2]
 *    (board/immutable_board.py:16-24); player 0 = PLAYER1, 1 = PLAYER2
 *    (types/moves.py:36-42).
 */
#ifndef BGX_H
#define BGX_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BGX_ABI_VERSION 10

#define BGX_OK 0
#define BGX_E_ARG -1        /* invalid argument */
#define BGX_E_HIP -2        /* HIP runtime error */
#define BGX_E_CAPACITY -3   /* a device buffer overflowed (see message) */
#define BGX_E_STATE -4      /* call not valid in the current state */

int bgx_abi_version(void);
const char* bgx_last_error(void);

/* Input domain of the stateless entry points below (bgx_movegen, bgx_encode,
 * bgx_value_boards, bgx_two_ply*): the boards a game can reach, as the
 * reference's ImmutableBoard holds them (board/immutable_board.py:16-24) —
 * every count <= 15, at most 15 checkers per player (points + bar + off), no
 * point held by both players — player 0 / 1 and dice 1..6 (randint(1, 7),
 * environments/backgammon_env.py:310-311). The check runs on the device (the
 * inputs stay device pointers); an input outside it makes the call return
 * BGX_E_ARG with the offending bits and the first bad index in the message,
 * before any output is written. These calls therefore synchronize `stream`
 * once (the reference's move_checker only prints a warning on an invalid move,
 * immutable_board.py:197-236; here nothing is computed for such a batch). */
#define BGX_BADF_SHARED_POINT 1u   /* a point holds checkers of both players */
#define BGX_BADF_TOTAL 2u          /* a player has more than 15 checkers */
#define BGX_BADF_VALUE 4u          /* a board byte above 15 */
#define BGX_BADF_DICE 8u           /* a die outside 1..6 */
#define BGX_BADF_PLAYER 16u        /* a player byte other than 0 / 1 */

/* The same check on its own: *h_flags = OR of BGX_BADF_* over the n inputs,
 * *h_first_bad = the lowest offending index (-1 if none). d_player and d_dice
 * may be NULL (not checked). Returns BGX_OK whatever the flags; synchronizes. */
int bgx_check_boards(const uint8_t* d_boards, const uint8_t* d_player, const uint8_t* d_dice, int n,
                     uint32_t* h_flags, int32_t* h_first_bad, void* stream);
/* The same rule on host arrays (no device; the host variant of the check). */
int bgx_check_boards_host(const uint8_t* h_boards, const uint8_t* h_player, const uint8_t* h_dice, int n,
                          uint32_t* h_flags, int32_t* h_first_bad);

/* ---------------- stateless parity entry points ---------------- */

/* get_all_possible_moves (backgammon/moves/generate_all_moves.py:7-90) for n
 * (board, player, dice) jobs, followed by execute_full_move_on_board_copy of
 * every FullMove (environments/env_helper.py:27-91): d_out_boards[j][k] (u8[52])
 * is the k-th result board of job j in the reference's order, for k < cap;
 * d_out_count[j] is the full number of results (may exceed cap). */
int bgx_movegen(const uint8_t* d_boards, const uint8_t* d_player, const uint8_t* d_dice, int n,
                uint8_t* d_out_boards, int32_t* d_out_count, int cap, void* stream);

/* ImmutableBoard.get_board_features (board/immutable_board.py:86-128) for
 * layout 0, generate_board_tensor.compute_features (:98-140) for layout 1;
 * d_out is float32 [n][198]. */
int bgx_encode(const uint8_t* d_boards, const uint8_t* d_player, int n, float* d_out, int layout,
               void* stream);

/* bgx_encode on the engine's own packed boards (bgx_harvest records and
 * headers, u32[8] each; the indicator player in word 6): for the callers that
 * re-encode harvested observations (Episode.observation / next_observation,
 * the trainer's inputs). Such boards come from the engine, so there is no
 * input-domain check and no synchronization: asynchronous on `stream`, and
 * capturable in a stream graph. Same values as bgx_encode of the unpacked
 * board. */
int bgx_encode_packed(const uint32_t* d_packed, int n, float* d_out, int layout, void* stream);

/* ---------------- value network ---------------- */
typedef struct bgx_net bgx_net;

/* BackgammonPolicyNetwork (agents/policy_network.py:36-70) weights, host fp32:
 * h_W1 [128][198] (fc1.weight), h_b1 [128], h_w2 [128] (value_head.weight), h_b2 [1]. */
int bgx_net_create(const float* h_W1, const float* h_b1, const float* h_w2, const float* h_b2,
                   bgx_net** out);
int bgx_net_destroy(bgx_net* net);
/* forward (policy_network.py:53-70) on arbitrary fp32 features d_x [n][198] -> d_out [n] */
int bgx_value(const bgx_net* net, const float* d_x, int n, float* d_out, void* stream);
/* fused encode + forward on boards (the engine's MFMA path): V of
 * get_board_features(board, player) for n boards -> d_out [n] */
int bgx_value_boards(const bgx_net* net, const uint8_t* d_boards, const uint8_t* d_player, int n,
                     float* d_out, void* stream);

/* compute_weighted_opponent_response (multi/two_ply.py:93-150) in exact mode
 * (no random.sample of 1-1/2-2/3-3 replies): for n afterstates d_boards and
 * the player to reply d_opponent, d_out[i] = sum over the 21 rolls of
 * P(roll) * mean of the top-5 V of the opponent's replies (V with the
 * opponent's indicator). Synchronizes `stream`. */
int bgx_two_ply(const bgx_net* net, const uint8_t* d_boards, const uint8_t* d_opponent, int n,
                double* d_out, void* stream);

/* bgx_two_ply in the reference-sampled mode (multi/two_ply.py:119-121): for
 * the rolls 1-1, 2-2 and 3-3 a reply set larger than sample_k (the reference:
 * 50) is replaced by a uniformly random sample_k of its replies
 * (random.sample; here a keyed permutation, reproducible per seed) before the
 * top-5 mean. sample_k = 0 is the exact mode (= bgx_two_ply). */
int bgx_two_ply_sampled(const bgx_net* net, const uint8_t* d_boards, const uint8_t* d_opponent, int n,
                        int sample_k, uint64_t seed, double* d_out, void* stream);

/* ---------------- self-play engine ---------------- */
typedef struct bgx_engine bgx_engine;

typedef struct bgx_config {
    int lanes;              /* game lanes on this device */
    int lane_base;          /* global id of lane 0 (RNG streams keyed by global lane id) */
    uint64_t seed;
    int ply;                /* 1 = worker.py:78-174 softmax(V/T); 2 = two_ply.py scoring */
    int k_top;              /* 2-ply candidates: 4 (reference, two_ply.py:67-70) or 0 = all */
    float alpha, beta;      /* 2-ply score = alpha*S - beta*W (two_ply.py:44-50): 1.0, 0.9 */
    int max_steps;          /* MAX_TIMESTEPS (config/configuration.py:4): 300 (at most 511) */
    int max_legal;          /* BackgammonEnv max_legal_moves (backgammon_env.py:35): 500; at most 512
                               (phased engine) or 2048 (fused 1-ply engine) */
    int ring;               /* experience ring slots per lane (>= max_steps + steps between harvests;
                               rounded up to a power of two; default 1024) */
    int ep_cap;             /* finished-episode headers held between harvests (0 = derived: every
                               episode that can finish in ring - max_steps steps) */
    int cand_per_lane;      /* average candidate rows reserved per lane (1-ply buffer) */
    int reply_per_lane;     /* average 2-ply reply rows reserved per lane */
    int greedy;             /* 1: argmax of the scores instead of sampling (play_versus_ai.py:188-195,
                               torch.argmax: first maximum); the sampling uniform is still drawn */
    int fused;              /* 1-ply only, 1 (default): bgx_step runs as ONE persistent launch in which
                               each workgroup (one per CU: 32 lanes on 12 waves when lanes >= 32 x CUs,
                               else 16 lanes on 8 waves) advances its lanes through all n_steps
                               (movegen, MLP, select, step fused; same results as 0 = one launch per
                               phase) */
    int reply_sample;       /* 2-ply: 0 (default) = exact mode; 50 = the reference's random.sample of 50
                               replies for 1-1 / 2-2 / 3-3 (two_ply.py:119-121), keyed by seed + step */
    int balance;            /* fused 1-ply, lanes <= 32 x CUs: 1 = bgx_step(n) runs n x lanes lane-steps in
                               total instead of n steps of every lane: the workgroups whose lanes step
                               faster run ahead (a lane may run up to n + n/4 + 4 steps in a call, at most
                               ring - max_steps), so a launch does not wait for its slowest workgroup.
                               Each lane's game is unchanged (dice and sampling keyed by lane and its own
                               counters), as the reference's 7 workers each run at their own pace
                               (main.py:86-91); only how far each lane got at a harvest differs.
                               0 (default) = lockstep. */
} bgx_config;

void bgx_config_default(bgx_config* cfg);

/* Replaces the per-process Worker (multi/worker.py:17-45) + BackgammonEnv
 * (environments/backgammon_env.py:29-128): `lanes` independent games on one
 * device, all reset per BackgammonEnv.reset. */
int bgx_engine_create(int device, const bgx_config* cfg, bgx_engine** out);
int bgx_engine_destroy(bgx_engine* e);

/* ParameterManager.get_parameters / get_temperature hand-off
 * (multi/parameter_manager.py:54-111, worker.py:66-76): host fp32 weights as
 * in bgx_net_create, the sampling temperature and the parameter version. */
int bgx_set_weights(bgx_engine* e, const float* h_W1, const float* h_b1, const float* h_w2,
                    const float* h_b2, float temperature, uint64_t version);

/* Test hook for parity replays: scripted dice. h_dice (host) holds, per lane,
 * per_lane single-die draws (1..6) that replace np.random.randint(1, 7)
 * (backgammon_env.py:310-311): every roll takes the lane's next two, starting
 * with BackgammonEnv.reset's starter and first rolls (backgammon_env.py:92-128).
 * Needs cfg.greedy (no sampling uniform is drawn); every lane restarts from
 * the reset. Reading past a lane's draws raises BGX_E_CAPACITY at the next
 * bgx_sync / bgx_harvest (the roll is then 1-2). */
int bgx_engine_set_dice(bgx_engine* e, const uint8_t* h_dice, int per_lane);

/* Advance every lane by n_steps env steps (one BackgammonEnv.step each,
 * passes included; finished games are recorded and the lane restarts); with
 * cfg.balance, n_steps x lanes lane-steps in total (bgx_get_stats counts them). */
int bgx_step(bgx_engine* e, int n_steps, void* stream);
/* Wait for the engine's stream; reports device-side overflow flags. */
int bgx_sync(bgx_engine* e);

/* Finished episodes since the last harvest (Episode/Experience,
 * environments/episode.py:5-84). Both arrays are DEVICE memory owned by the
 * engine, valid until the second bgx_harvest after this one; each episode's records
 * are contiguous, in header order:
 *   headers [n_episodes][16] u32: global lane, episode no., first record,
 *     n_records, env steps, win_type | winner << 8 | flags << 16, the final
 *     board (packed words 0..6), 0, 0, 0
 *   records [n_records][12] u32 (48 B): the board before the move (packed
 *     words 0..6; the indicator = the mover), V(s) f32, V(a) f32, reward f32,
 *     action | n_moves << 11 | step << 23 (n_moves saturates at 4095),
 *     dice0 | dice1 << 3 | done << 6 | close_out << 7 | prime << 8 |
 *     mover << 9 | win_type << 10.
 * The board after record k's move (Experience.next_observation) is record
 * k+1's before-board (passes move no checker), and for an episode's last
 * record the header's final board; its indicator is the mover at a terminal
 * step (the winner), else the other player (backgammon_env.py:196-218).
 * Packed board: u32[8]: P1 point nibbles [0..2], P2 [3..5], w[6] = bar1 |
 * bar2 << 4 | off1 << 8 | off2 << 12 | indicator player << 16.
 * Synchronizes the engine stream. */
typedef struct bgx_harvest_info {
    int n_episodes;
    int n_records;
    const uint32_t* d_headers;
    const uint32_t* d_records;
} bgx_harvest_info;
int bgx_harvest(bgx_engine* e, bgx_harvest_info* out, void* stream);

/* bgx_harvest in two halves, so the host does not stall the device between
 * steps: bgx_harvest_enqueue queues the harvest on `stream` (behind the
 * engine's last step; the next bgx_step waits for it) and returns a ticket at
 * once; bgx_harvest_fetch(ticket) waits for that harvest and fills `out` as
 * bgx_harvest does. Three buffers rotate: a ticket's arrays stay valid until
 * the second bgx_harvest_enqueue after it, and only the last two tickets can
 * be fetched. (bgx_harvest = enqueue + fetch.) A fused 1-ply engine harvests
 * inside its step launches (each workgroup its own lanes, into the buffer of
 * the next ticket), so enqueue only records the point; the contract is the
 * same. */
int bgx_harvest_enqueue(bgx_engine* e, int* ticket, void* stream);
int bgx_harvest_fetch(bgx_engine* e, int ticket, bgx_harvest_info* out);
/* Error flags (capacity overflows, a bounded wait) belong to a ticket: the
 * device moves the flags raised by the steps since the previous ticket into
 * that ticket's totals (an atomic exchange, in stream order), and
 * bgx_harvest_fetch reports them for that ticket only; a launch in flight
 * during the fetch is never affected. bgx_sync reports the flags raised since
 * the last ticket. A fused engine's workgroup whose finished episodes do not
 * fit the ticket's output copies nothing and keeps them in its lanes' rings
 * for the next ticket (not an error); episodes are lost, and reported, only
 * when a lane's ring is overwritten before they are harvested. */

typedef struct bgx_stats {
    uint64_t env_steps;     /* lane steps (passes included) */
    uint64_t decisions;     /* non-pass steps (one Experience each) */
    uint64_t episodes;
    uint64_t value_rows;    /* boards evaluated by the value MLP */
    uint64_t movegen_jobs;  /* (board, dice) move generations */
    uint64_t fallback_jobs; /* doubles jobs re-run on the global-memory path */
    uint64_t gap_rows;      /* of value_rows: 2-ply reply rows reserved in per-wave chunks but left
                               unwritten (the reply MLP evaluates them; no record reads them) */
} bgx_stats;
int bgx_get_stats(bgx_engine* e, bgx_stats* out);  /* synchronizes */

/* Test hook: copy one of the phased engine's per-step device buffers to host
 * (synchronizes the engine stream), so a parity test can compare what a
 * bgx_step computed at the benchmarked shape with the oracle. After a step:
 * the candidates of that step (their rows, per-lane offset / count, V) and,
 * at ply 2, the top-k choice and the per-(candidate, roll) top-5 reply means
 * that two_ply.py:93-150 averages into W (job (candidate row - L) * 21 + roll
 * at K = all, (4 * lane + k) * 21 + roll at K = 4; DICE_ROLLS order,
 * two_ply.py:10-32). Before a step: the lanes' boards, players and dice.
 * h_out = null returns the size in *needed only. The fused 1-ply engine keeps
 * its candidates in workgroup-private buffers: only PLAYER / DICE there. */
enum {
    BGX_PEEK_LANE_ROWS = 0,   /* u32 [L][8] packed lane boards */
    BGX_PEEK_PLAYER = 1,      /* u8 [L] player to move */
    BGX_PEEK_DICE = 2,        /* u8 [L][2] the roll to play */
    BGX_PEEK_CAND_OFF = 3,    /* i32 [L] first candidate row (after row L) */
    BGX_PEEK_CAND_CNT = 4,    /* i32 [L] candidates (all, before the max_legal cap) */
    BGX_PEEK_CAND_ROWS = 5,   /* u32 [cand_cap][8] packed candidate boards */
    BGX_PEEK_VALUES = 6,      /* f32 [L + cand_cap] V of the lane rows, then of the candidates */
    BGX_PEEK_SEL = 7,         /* i32 [L][4] K = 4: the chosen candidate rows (-1: fewer than 4 moves) */
    BGX_PEEK_JOB_VAL = 8      /* f32 [jobs] top-5 mean of the replies per (candidate, roll) */
};
int bgx_engine_peek(bgx_engine* e, int buf, void* h_out, uint64_t bytes, uint64_t* needed);

/* Kernel timing (HIP events on the engine stream, recorded per bgx_step while
 * enabled): total milliseconds and launch counts of the movegen and MLP
 * kernels since the last reset. A fused engine (bgx_config.fused, 1-ply)
 * reports its one step kernel (all n_steps of a bgx_step) in the movegen slot
 * and 0 MLP launches. */
int bgx_set_timing(bgx_engine* e, int enabled);
int bgx_get_timing(bgx_engine* e, double* ms_movegen, int* n_movegen, double* ms_mlp, int* n_mlp);

/* TD(0) update on the device: replaces Trainer.update's
 * per-episode loop (src/agents/trainer.py:81-138: forward, TD(0) target with
 * gamma * V[t+1] detached, MSE, backward, clip_grad_norm_(clip), Adam step)
 * with one launch over n_eps episodes of bgx_harvest records (episode e =
 * records [d_offs[e], d_offs[e+1]), at most 2048 each). d_params / d_adam_m /
 * d_adam_v: 25,729 fp32 each in state_dict order (fc1.weight [128][198],
 * fc1.bias, value_head.weight, value_head.bias), updated in place; *d_step =
 * Adam's step count (incremented per episode); d_metrics[5] (double) +=
 * per-episode loss, post-clip grad norm, mean |TD error|, mean V, reward sum.
 * grad_clip <= 0: no clipping. Asynchronous on `stream`. */
int bgx_td0_update(const uint32_t* d_records, const int32_t* d_offs, int n_eps, float* d_params,
                   float* d_adam_m, float* d_adam_v, int* d_step, float lr, float gamma, float grad_clip,
                   double* d_metrics, void* stream);

/* Copy-engine transfer helpers (bgx/hostgather.py: the episode gather of
 * the ranks of one node through host shared memory, replacing the pickled
 * queue of src/main.py:115-133 / multi/experience_queue.py:5-13 without
 * using compute units): page-lock an existing host range (a shared-memory
 * segment) for DMA, and an asynchronous copy between any two of device /
 * page-locked host memory on `stream` (hipMemcpyAsync, hipMemcpyDefault:
 * DMA engines, no kernel). */
int bgx_host_register(void* h_ptr, uint64_t bytes);
int bgx_host_unregister(void* h_ptr);
int bgx_copy_async(void* dst, const void* src, uint64_t bytes, int kind, void* stream);   /* kind: 0 default
                                  (inferred), 1 host->device, 2 device->host, 3 device->device, 4 device->device
                                  on the DMA engines (hipMemcpyDeviceToDeviceNoCU; also into page-locked host
                                  memory, which the device addresses directly) */

/* Device -> host copy on a DMA engine (SDMA, through the HSA runtime; the
 * HIP runtime here serves such copies with blit kernels, which need compute
 * units and queue behind a persistent kernel). h_dst must lie in a range
 * page-locked with bgx_host_register; the copy starts at once (the caller has
 * made d_src ready, e.g. by bgx_harvest_fetch) and *ticket identifies it;
 * bgx_dma_wait(ticket, timeout_ms <= 0: no limit) waits for it and releases the
 * ticket (exactly once per ticket). BGX_E_STATE when the device has no DMA
 * engine for the direction, or when the wait times out: the copy is then still
 * in flight, the ticket stays valid (wait again) and both buffers must stay
 * allocated until a wait succeeds. */
int bgx_dma_copy_d2h(void* h_dst, const void* d_src, uint64_t bytes, int device, uint64_t* ticket);
int bgx_dma_wait(uint64_t ticket, int timeout_ms);

/* Device -> device copy on a DMA engine of the source GPU (SDMA through the HSA
 * runtime; over xGMI when the destination is another GPU's memory, e.g. a
 * range of the trainer rank's GPU opened with bgx_ipc_open). d_dst lies in
 * device memory of GPU dst_device (as this process numbers the GPUs), d_src in
 * GPU src_device's. Waited for with bgx_dma_wait. Replaces, for the device
 * hand-off of bgx/devgather.py, the reference's pickled Queue hand-off of
 * finished Episodes (src/main.py:115-133, multi/experience_queue.py:5-13)
 * whose consumer moves them to the trainer's device (main.py:129-133). */
int bgx_dma_copy_d2d(void* d_dst, int dst_device, const void* d_src, int src_device, uint64_t bytes,
                     uint64_t* ticket);

/* Inter-process access to device memory (one process per GPU): export a
 * range (handle of its allocation + the offset of d_ptr in it), open it in
 * another process (mapped on this process's current device, peer access
 * enabled), close it. */
int bgx_ipc_export(const void* d_ptr, uint8_t* handle64, uint64_t* offset);
int bgx_ipc_open(const uint8_t* handle64, uint64_t offset, void** d_ptr);
int bgx_ipc_close(void* d_ptr, uint64_t offset);

/* The 2-ply reply expansion alone (the engine's and bgx_two_ply's reply
 * launch, two_ply.py:114-133 before the value calls): for each of n candidate
 * boards, the opponent's legal afterstates for all 21 DICE_ROLLS
 * (two_ply.py:10-32), as packed boards (flag = the opponent) in d_out[cap][8];
 * job i * 21 + r's records are rows d_off[j] .. d_off[j] + d_cnt[j] - 1
 * (other rows are unused). Parity hook for the board-major reply kernel
 * (BGX_REPLY_BM=0 selects the per-(board, roll) kernel); BGX_E_CAPACITY when
 * cap is too small. Rows are reserved in chunks per workgroup, so cap needs
 * slack beyond the records: per workgroup of the launch (min(2 x CUs,
 * ceil(7 n / 16)) workgroups) its last chunk's unwritten tail (<= 2,048 rows)
 * and its waves' kept remainders (each smaller than one job's records);
 * bgx/ops.py reply_moves allows 4,096 rows per workgroup. */
int bgx_reply_moves(const uint8_t* d_boards, const uint8_t* d_opponent, int n, uint32_t* d_out, int cap,
                    int32_t* d_off, int32_t* d_cnt, void* stream);

/* Convert between u8[52] boards and the engine's packed boards (device). */
int bgx_pack(const uint8_t* d_boards, const uint8_t* d_player, int n, uint32_t* d_packed, void* stream);
int bgx_unpack(const uint32_t* d_packed, int n, uint8_t* d_boards, void* stream);

#ifdef __cplusplus
}
#endif
#endif
