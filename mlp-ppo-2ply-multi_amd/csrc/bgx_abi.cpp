// bgx_abi.cpp — the extern "C" boundary of libbgx.so (declared in include/bgx.h).
//
// Host-side orchestration only: argument checks, device buffers, the
// per-step launch sequence and error reporting. All game logic runs in the
// HIP kernels (bgx_movegen.hip, bgx_mlp.hip, bgx_encode.hip, bgx_engine.hip).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <cstdlib>
#include <exception>
#include <new>
#include <algorithm>
#include <chrono>
#include <mutex>
#include <vector>

#include "bgx.h"
#include "bgx_domain.h"
#include "bgx_frag.h"
#include "bgx_kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess)                                                             \
            return fail(BGX_E_HIP, "%s failed: %s", #expr, hipGetErrorString(_e));       \
    } while (0)

using bgx_frag::build_fragments;
using bgx_frag::KSTEPS;
using bgx_frag::NFRAG;

template <typename T>
int dalloc(T** p, size_t n) {
    hipError_t e = hipMalloc((void**)p, n * sizeof(T) + 16);
    if (e != hipSuccess) return fail(BGX_E_HIP, "hipMalloc(%zu B): %s", n * sizeof(T), hipGetErrorString(e));
    return BGX_OK;
}

}  // namespace

struct bgx_net {
    float* W1 = nullptr;   // fp32 copies (bgx_value)
    float* b1 = nullptr;
    float* w2 = nullptr;
    float b2 = 0.0f;
    uint4* wfrag = nullptr;   // split-fp16 MFMA fragments
    float* rowc = nullptr;    // [128] w2
    float feat_scale = 1.0f;  // 2^-e: features scaled so the accumulator is the exp2 argument
};

static int net_upload(bgx_net* n, const float* W1, const float* b1, const float* w2, const float* b2) {
    std::vector<uint16_t> frag;
    const int e = build_fragments(W1, b1, frag);
    n->feat_scale = (float)std::ldexp(1.0, -e);
    HIP_TRY(hipMemcpy(n->W1, W1, 128 * 198 * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(n->b1, b1, 128 * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(n->w2, w2, 128 * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(n->wfrag, frag.data(), frag.size() * 2, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(n->rowc, w2, 128 * 4, hipMemcpyHostToDevice));
    n->b2 = b2[0];
    return BGX_OK;
}

constexpr int PROF_W = 128;   // u64 words per workgroup slot of the fused development report (bgx_fused.hip PROF_STRIDE)

struct bgx_engine {
    int device = 0;
    bgx_config cfg{};
    bgx_net* net = nullptr;
    bgx::EngineDev d{};
    hipStream_t last = nullptr;
    // device buffers
    uint32_t* rows = nullptr;
    float* V = nullptr;
    int32_t* cand_off = nullptr;
    int32_t* cand_cnt = nullptr;
    unsigned* ctr = nullptr;   // [3] ep, [4] err; per-step (zeroed each step): [8] flat, [9] reply, [10] ovf, [11] ovf2;
                               // [12..15] balanced-launch counters (lane-steps, finished workgroups)
    unsigned long long* stats = nullptr;
    int32_t* sel = nullptr;
    uint32_t* sel_rows = nullptr;
    uint32_t* reply_rows = nullptr;
    float* reply_V = nullptr;
    int32_t* job_off = nullptr;
    int32_t* job_cnt = nullptr;
    float* job_val = nullptr;
    float* zt = nullptr;            // 2-ply: the reply roots' hidden accumulators [roots][128] (K = all: every
                                    // candidate, from the root launch; K = 4: the chosen rows, own launch)
    float* zv = nullptr;            // K = 4: that launch's V output (unused)
    int jobs_cap = 0, reply_cap = 0, cand_cap = 0;
    int32_t* ovf_list = nullptr;
    int ovf_cap = 0;
    uint32_t* ws = nullptr;
    int ws_waves = 0, ws_slots = 0;
    // fused 1-ply step: per-lane candidate slots and values
    bool fused = false;
    uint32_t* fcand = nullptr;
    float* fvbuf = nullptr;
    int* ft1cnt = nullptr;   // fused: the lanes' next-position expansion counts (FusedArgs::t1cnt)
    bool t1_ready = false;   // ... valid: set by a fused launch, cleared by every lane reset
    int fcap = 0;
    unsigned long long* fprof = nullptr;   // BGX_FUSED_PROF: phase clocks, printed at destroy
    // harvest: records of at most L x ring (every unharvested record of every lane)
    // three harvest buffers (bgx_harvest_enqueue / _fetch): ticket t uses slot
    // t % 3. A ticket's arrays live until the second harvest after it; the
    // fused engine harvests inside its launches, so the launches between
    // tickets t + 1 and t + 2 already fill slot (t + 2) % 3: a third slot keeps
    // ticket t's arrays intact until then
    static constexpr int NHB = 3;
    uint32_t* out_records[NHB] = {nullptr, nullptr, nullptr};
    uint32_t* out_headers[NHB] = {nullptr, nullptr, nullptr};   // [ep_cap][16] copies of the finished episodes' headers
    int32_t* d_offs[NHB] = {nullptr, nullptr, nullptr};     // [ep_cap + 1]
    uint32_t* d_info[NHB] = {nullptr, nullptr, nullptr};    // [4] harvest totals
    uint32_t* h_info = nullptr;    // [NHB][4] host-mapped copies, written by the harvesting kernel itself
    uint32_t* h_info_dev = nullptr;   // its device address
    // fused engine (in-kernel harvest): per slot the running {episodes << 32 |
    // records} appended since the previous ticket, [NHB] = finished workgroups,
    // [NHB + 1 + b] = slot b's accumulated error flags (moved there from the
    // engine's word by each launch's last workgroup)
    unsigned long long* fh_ctr = nullptr;
    bool fh_launched = false;      // a fused launch filled the current slot since the last ticket
    hipEvent_t hev = nullptr;         // the engine's last step, for a harvest on another stream
    hipEvent_t hdone[NHB] = {nullptr, nullptr, nullptr};   // a slot's harvest finished
    hipStream_t hstream = nullptr;    // stream of the last enqueued harvest (the next step waits for it)
    int h_tickets = 0;                // harvests enqueued so far
    // timing
    bool timing = false;
    std::vector<hipEvent_t> ev;   // pairs: movegen, mlp
    // test / development hooks, read once at create: BGX_MG_TEST_TIER (fused
    // movegen tiers), BGX_FUSED_PROF (phase clocks, printed at destroy)
    int force_tier = 0;
    bool prof_enabled = false;
    int fused_fl = 0;             // BGX_FUSED_LANES: fused 1-ply lanes per workgroup (16 / 32; 0 = auto)
    uint8_t* dice_tab = nullptr;  // bgx_engine_set_dice
    std::vector<int> ev_kind;
    double ms_mg = 0, ms_mlp = 0;
    int n_mg = 0, n_mlp = 0;
    // optional hipGraph of the last n_steps sequence
    bool use_graph = false;   // measured slower than direct launches on ROCm 7 (BGX_GRAPH=1 enables)
    hipStream_t cap = nullptr;
    hipGraphExec_t gexec = nullptr;
    int g_steps = 0;
};

namespace {
constexpr int C_EP = 3, C_ERR = 4, C_FLAT = 8, C_REPLY = 9, C_OVF = 10, C_OVF2 = 11;
// stats words: [0..7] counters (bgx_get_stats), then the top-5 launch's per-wave
// reply-record counts
constexpr int kStatWords = 8 + bgx::T5_WAVES;
constexpr int C_BUDGET = 12;   // [12..15]: the balanced fused launch's lane-step and finished-workgroup counters (u64)
}

static int flag_error(unsigned f) {
    return fail(f & BGX_ERRF_WAIT_BOUND ? BGX_E_STATE : BGX_E_CAPACITY,
                "device flags 0x%x (1 flat rows, 2 overflow list, 4 fallback workspace, 8 experience ring, "
                "16 episode list, 32 scripted dice: capacity; 64 an intra-workgroup wait hit its bound: state)", f);
}

// after the engine's stream is synchronized: the flags raised since the last
// harvest ticket (they move into a ticket's totals when it is harvested, and
// bgx_harvest_fetch reports them there). The engine word is reset here; a
// fused engine's launches have already moved theirs into the open ticket's
// accumulator, which is reported but left for the ticket.
static int check_flags(bgx_engine* e) {
    unsigned f = 0;
    HIP_TRY(hipMemcpy(&f, e->ctr + C_ERR, 4, hipMemcpyDeviceToHost));
    if (f) HIP_TRY(hipMemset(e->ctr + C_ERR, 0, 4));
    if (e->fh_ctr) {
        unsigned long long acc = 0;
        HIP_TRY(hipMemcpy(&acc, e->fh_ctr + bgx_engine::NHB + 1 + e->h_tickets % bgx_engine::NHB, 8,
                          hipMemcpyDeviceToHost));
        f |= (unsigned)acc;
    }
    return f ? flag_error(f) : BGX_OK;
}


// Every int entry point runs inside guarded(): a C++ exception (std::bad_alloc
// from a host vector, ...) becomes an error code and bgx_last_error(), never an
// unwind across the C boundary.
template <typename F>
static int guarded(const char* what, F&& body) noexcept {
    try {
        return body();
    } catch (const std::bad_alloc&) {
        return fail(BGX_E_CAPACITY, "%s: host allocation failed", what);
    } catch (const std::exception& ex) {
        return fail(BGX_E_STATE, "%s: %s", what, ex.what());
    } catch (...) {
        return fail(BGX_E_STATE, "%s: unexpected C++ exception", what);
    }
}

// ---------------------------------------------------------------- stateless-call scratch
// The stateless entry points need a few device words (validation flags,
// movegen overflow counters), an overflow list, a fallback workspace and (for
// bgx_value_boards) packed boards. Each call leases one scratch set from a
// per-device pool: a set is handed out only when no call holds it and the
// stream work of its last user has finished (an event recorded at release),
// so calls from several host threads or on several streams never share one.
// Sets are kept for reuse; the pool grows to the peak number of calls in flight.
namespace {

struct Scratch {
    int dev = -1;
    bool busy = false;
    hipEvent_t done = nullptr;
    unsigned* words = nullptr;     // [16]: [0..1] validation flags, [2] ovf count, [3] err flags
    uint32_t* h_words = nullptr;   // pinned host copy of words[0..1]
    int32_t* ovf = nullptr;        // movegen overflow list (lazy)
    uint32_t* ws = nullptr;        // movegen fallback workspace (lazy)
    uint32_t* packed = nullptr;    // bgx_value_boards packed boards (lazy, grows)
    size_t packed_n = 0;
};

constexpr int SC_OVF_CAP = 1 << 16, SC_WS_WAVES = 256, SC_WS_SLOTS = 16384;

std::mutex g_pool_mu;
std::vector<Scratch*> g_pool;

// hipSetDevice to the device holding `p` (a device pointer) for the scope; the
// caller's current device is restored at the end
struct DeviceScope {
    int prev = -1;
    int dev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceScope(const void* p) {
        err = hipGetDevice(&prev);
        if (err != hipSuccess) return;
        dev = prev;
        hipPointerAttribute_t at{};
        if (p && hipPointerGetAttributes(&at, p) == hipSuccess && at.device >= 0 && at.device != prev) {
            err = hipSetDevice(at.device);
            dev = at.device;
        }
        (void)hipGetLastError();   // a host pointer's attribute query is not an error here
    }
    ~DeviceScope() {
        if (prev >= 0 && dev != prev) (void)hipSetDevice(prev);
    }
};

struct Lease {
    Scratch* sc = nullptr;
    hipStream_t stream = nullptr;
    ~Lease() {
        if (!sc) return;
        (void)hipEventRecord(sc->done, stream);
        std::lock_guard<std::mutex> g(g_pool_mu);
        sc->busy = false;
    }
};

int lease_scratch(hipStream_t stream, Lease& L) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (Scratch* sc : g_pool) {
            if (sc->dev != dev || sc->busy || hipEventQuery(sc->done) != hipSuccess) continue;
            sc->busy = true;
            L.sc = sc;
            L.stream = stream;
            return BGX_OK;
        }
    }
    Scratch* sc = new Scratch();
    sc->dev = dev;
    sc->busy = true;
    if (dalloc(&sc->words, 16)) {
        delete sc;
        return BGX_E_HIP;
    }
    if (hipHostMalloc((void**)&sc->h_words, 4 * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&sc->done, hipEventDisableTiming) != hipSuccess) {
        hipFree(sc->words);
        if (sc->h_words) hipHostFree(sc->h_words);
        delete sc;
        return fail(BGX_E_HIP, "scratch: pinned buffer / event creation failed");
    }
    HIP_TRY(hipMemset(sc->words, 0, 64));
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        g_pool.push_back(sc);
    }
    L.sc = sc;
    L.stream = stream;
    return BGX_OK;
}

int lease_movegen_space(Scratch* sc) {
    if (!sc->ovf && dalloc(&sc->ovf, SC_OVF_CAP)) return BGX_E_HIP;
    if (!sc->ws && dalloc(&sc->ws, (size_t)SC_WS_WAVES * 5 * SC_WS_SLOTS)) return BGX_E_HIP;
    return BGX_OK;
}

// the input-domain check (include/bgx.h, BGX_BADF_*): flags into the lease's
// words, copied to pinned memory, one stream synchronization
int check_domain(Scratch* sc, const uint8_t* boards, const uint8_t* player, const uint8_t* dice, int n,
                 hipStream_t s, uint32_t* flags, int32_t* first) {
    HIP_TRY(bgx_launch_validate(boards, player, dice, n, sc->words, s));
    HIP_TRY(hipMemcpyAsync(sc->h_words, sc->words, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *flags = sc->h_words[0];
    *first = sc->h_words[0] ? (int32_t)sc->h_words[1] : -1;
    return BGX_OK;
}

int require_domain(const char* what, Scratch* sc, const uint8_t* boards, const uint8_t* player,
                   const uint8_t* dice, int n, hipStream_t s) {
    uint32_t f = 0;
    int32_t first = -1;
    if (int rc = check_domain(sc, boards, player, dice, n, s, &f, &first)) return rc;
    if (f)
        return fail(BGX_E_ARG,
                    "%s: input %d is outside the board domain (bits 0x%x: 1 a point held by both players, 2 more "
                    "than 15 checkers of a player, 4 a count above 15, 8 a die outside 1..6, 16 a player not 0/1)",
                    what, first, f);
    return BGX_OK;
}

}  // namespace

// ---- DMA-engine copies (SDMA through the HSA runtime). On this ROCm the HIP
// runtime serves device <-> host hipMemcpyAsync with blit kernels, which need
// compute units and so queue behind a persistent kernel; these copies go to a
// DMA engine explicitly (hsa_amd_memory_async_copy_on_engine, forced SDMA).
namespace {
struct DmaDev {
    bool ready = false;
    hsa_agent_t gpu{}, cpu{};
    hsa_amd_sdma_engine_id_t engine = HSA_AMD_SDMA_ENGINE_0;
};
std::mutex g_dma_mu;
DmaDev g_dma[64];

struct AgentQuery {
    uint32_t bdf = 0, domain = 0;
    hsa_agent_t gpu{}, cpu{};
    bool have_gpu = false, have_cpu = false;
};

hsa_status_t find_agents(hsa_agent_t a, void* data) {
    AgentQuery* q = (AgentQuery*)data;
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_CPU && !q->have_cpu) {
        q->cpu = a;
        q->have_cpu = true;
    } else if (t == HSA_DEVICE_TYPE_GPU && !q->have_gpu) {
        uint32_t bdf = 0, dom = 0;
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
        if (bdf == q->bdf && dom == q->domain) {
            q->gpu = a;
            q->have_gpu = true;
        }
    }
    return HSA_STATUS_SUCCESS;
}

int dma_setup(int dev, DmaDev** out) {
    std::lock_guard<std::mutex> g(g_dma_mu);
    if (dev < 0 || dev >= 64) return fail(BGX_E_ARG, "bgx_dma: device %d", dev);
    DmaDev& d = g_dma[dev];
    if (!d.ready) {
        int bus = 0, slot = 0, dom = 0;
        HIP_TRY(hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, dev));
        HIP_TRY(hipDeviceGetAttribute(&slot, hipDeviceAttributePciDeviceId, dev));
        HIP_TRY(hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, dev));
        if (hsa_init() != HSA_STATUS_SUCCESS) return fail(BGX_E_STATE, "bgx_dma: hsa_init failed");
        AgentQuery q;
        q.bdf = ((uint32_t)bus << 8) | ((uint32_t)slot << 3);
        q.domain = (uint32_t)dom;
        hsa_iterate_agents(find_agents, &q);
        if (!q.have_gpu || !q.have_cpu) return fail(BGX_E_STATE, "bgx_dma: no HSA agent for device %d", dev);
        // the CPU agent of the GPU's own NUMA node (a multi-socket host lists one
        // CPU agent per node; the first one found may be the far socket)
        hsa_agent_t near{};
        if (hsa_agent_get_info(q.gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_NEAREST_CPU, &near) == HSA_STATUS_SUCCESS &&
            near.handle != 0)
            q.cpu = near;
        uint32_t mask = 0;
        if (hsa_amd_memory_copy_engine_status(q.cpu, q.gpu, &mask) != HSA_STATUS_SUCCESS || mask == 0)
            return fail(BGX_E_STATE, "bgx_dma: no DMA engine available for device %d -> host", dev);
        d.gpu = q.gpu;
        d.cpu = q.cpu;
        d.engine = (hsa_amd_sdma_engine_id_t)(mask & (~mask + 1u));   // the lowest available engine
        d.ready = true;
    }
    *out = &d;
    return BGX_OK;
}
}  // namespace

extern "C" {

int bgx_abi_version(void) { return BGX_ABI_VERSION; }
const char* bgx_last_error(void) { return g_err.c_str(); }

int bgx_check_boards_host(const uint8_t* h_boards, const uint8_t* h_player, const uint8_t* h_dice, int n,
                          uint32_t* h_flags, int32_t* h_first_bad) {
    return guarded("bgx_check_boards_host", [&]() -> int {
        if (n < 0 || !h_flags || !h_first_bad || (n > 0 && !h_boards))
            return fail(BGX_E_ARG, "bgx_check_boards_host: bad arguments (n=%d)", n);
        uint32_t f = 0;
        int32_t first = -1;
        for (int i = 0; i < n; ++i) {
            const unsigned b = bgx::domain_bits(h_boards + (size_t)i * 52, h_player ? (int)h_player[i] : -1,
                                                h_dice ? h_dice + 2 * (size_t)i : nullptr);
            if (b && first < 0) first = i;
            f |= b;
        }
        *h_flags = f;
        *h_first_bad = first;
        return BGX_OK;
    });
}

int bgx_check_boards(const uint8_t* d_boards, const uint8_t* d_player, const uint8_t* d_dice, int n,
                     uint32_t* h_flags, int32_t* h_first_bad, void* stream) {
    return guarded("bgx_check_boards", [&]() -> int {
        if (n < 0 || !h_flags || !h_first_bad || (n > 0 && !d_boards))
            return fail(BGX_E_ARG, "bgx_check_boards: bad arguments (n=%d)", n);
        *h_flags = 0;
        *h_first_bad = -1;
        if (n == 0) return BGX_OK;
        DeviceScope ds(d_boards);
        HIP_TRY(ds.err);
        Lease L;
        if (int rc = lease_scratch((hipStream_t)stream, L)) return rc;
        return check_domain(L.sc, d_boards, d_player, d_dice, n, (hipStream_t)stream, h_flags, h_first_bad);
    });
}

int bgx_movegen(const uint8_t* d_boards, const uint8_t* d_player, const uint8_t* d_dice, int n,
                uint8_t* d_out_boards, int32_t* d_out_count, int cap, void* stream) {
    return guarded("bgx_movegen", [&]() -> int {
        if (n < 0 || cap < 0) return fail(BGX_E_ARG, "bgx_movegen: n=%d cap=%d", n, cap);
        if (n == 0) return BGX_OK;
        if (!d_boards || !d_player || !d_dice || !d_out_count || (cap > 0 && !d_out_boards))
            return fail(BGX_E_ARG, "bgx_movegen: null pointer");
        DeviceScope ds(d_boards);
        HIP_TRY(ds.err);
        hipStream_t s = (hipStream_t)stream;
        Lease L;
        if (int rc = lease_scratch(s, L)) return rc;
        if (int rc = require_domain("bgx_movegen", L.sc, d_boards, d_player, d_dice, n, s)) return rc;
        if (int rc = lease_movegen_space(L.sc)) return rc;
        unsigned* ctr = L.sc->words + 2;   // [0] overflow count, [1] error flags
        bgx::MovegenArgs a{};
        a.n_jobs = n;
        a.in_mode = bgx::IN_U8;
        a.in_u8 = d_boards;
        a.in_player = d_player;
        a.in_dice = d_dice;
        a.out_mode = bgx::OUT_U8;
        a.cap = cap;
        a.out_u8 = d_out_boards;
        a.out_count = d_out_count;
        a.ovf_count = ctr;
        a.ovf_list = L.sc->ovf;
        a.ovf_cap = SC_OVF_CAP;
        a.ws_global = L.sc->ws;
        a.ws_waves = SC_WS_WAVES;
        a.ws_slots = SC_WS_SLOTS;
        a.ws_words_per_wave = (size_t)5 * SC_WS_SLOTS;
        a.err_flags = ctr + 1;
        HIP_TRY(bgx_launch_movegen(&a, s));
        return BGX_OK;
    });
}

int bgx_encode(const uint8_t* d_boards, const uint8_t* d_player, int n, float* d_out, int layout,
               void* stream) {
    return guarded("bgx_encode", [&]() -> int {
        if (n < 0 || (layout != 0 && layout != 1)) return fail(BGX_E_ARG, "bgx_encode: n=%d layout=%d", n, layout);
        if (n == 0) return BGX_OK;
        if (!d_boards || !d_player || !d_out) return fail(BGX_E_ARG, "bgx_encode: null pointer");
        DeviceScope ds(d_boards);
        HIP_TRY(ds.err);
        Lease L;
        if (int rc = lease_scratch((hipStream_t)stream, L)) return rc;
        if (int rc = require_domain("bgx_encode", L.sc, d_boards, d_player, nullptr, n, (hipStream_t)stream)) return rc;
        HIP_TRY(bgx_launch_encode(d_boards, d_player, n, d_out, layout, (hipStream_t)stream));
        return BGX_OK;
    });
}

int bgx_encode_packed(const uint32_t* d_packed, int n, float* d_out, int layout, void* stream) {
    return guarded("bgx_encode_packed", [&]() -> int {
        if (n < 0 || (layout != 0 && layout != 1))
            return fail(BGX_E_ARG, "bgx_encode_packed: n=%d layout=%d", n, layout);
        if (n == 0) return BGX_OK;
        if (!d_packed || !d_out) return fail(BGX_E_ARG, "bgx_encode_packed: null pointer");
        DeviceScope ds(d_packed);
        HIP_TRY(ds.err);
        HIP_TRY(bgx_launch_encode_packed(d_packed, n, d_out, layout, (hipStream_t)stream));
        return BGX_OK;
    });
}

int bgx_td0_update(const uint32_t* d_records, const int32_t* d_offs, int n_eps, float* d_params,
                   float* d_adam_m, float* d_adam_v, int* d_step, float lr, float gamma, float grad_clip,
                   double* d_metrics, void* stream) {
    return guarded("bgx_td0_update", [&]() -> int {
        if (n_eps < 0 || (n_eps > 0 && (!d_records || !d_offs || !d_params || !d_adam_m || !d_adam_v || !d_step ||
                                        !d_metrics)))
            return fail(BGX_E_ARG, "bgx_td0_update: bad arguments (n_eps=%d)", n_eps);
        DeviceScope ds(d_params);   // the kernel runs on the device holding the parameters
        HIP_TRY(ds.err);
        bgx::TrainArgs a{};
        a.rec = d_records;
        a.offs = d_offs;
        a.n_eps = n_eps;
        a.params = d_params;
        a.adam_m = d_adam_m;
        a.adam_v = d_adam_v;
        a.step = d_step;
        a.lr = lr;
        a.gamma = gamma;
        a.grad_clip = grad_clip;
        a.metrics = d_metrics;
        HIP_TRY(bgx_launch_td0(&a, (hipStream_t)stream));
        return BGX_OK;
    });
}

int bgx_host_register(void* h_ptr, uint64_t bytes) {
    return guarded("bgx_host_register", [&]() -> int {
        if (!h_ptr || bytes == 0) return fail(BGX_E_ARG, "bgx_host_register: bad arguments");
        HIP_TRY(hipHostRegister(h_ptr, (size_t)bytes, hipHostRegisterPortable));
        return BGX_OK;
    });
}

int bgx_host_unregister(void* h_ptr) {
    return guarded("bgx_host_unregister", [&]() -> int {
        if (!h_ptr) return fail(BGX_E_ARG, "bgx_host_unregister: null pointer");
        HIP_TRY(hipHostUnregister(h_ptr));
        return BGX_OK;
    });
}

int bgx_copy_async(void* dst, const void* src, uint64_t bytes, int kind, void* stream) {
    return guarded("bgx_copy_async", [&]() -> int {
        if (bytes == 0) return BGX_OK;
        if (!dst || !src || kind < 0 || kind > 4) return fail(BGX_E_ARG, "bgx_copy_async: bad arguments");
        const hipMemcpyKind k[5] = {hipMemcpyDefault, hipMemcpyHostToDevice, hipMemcpyDeviceToHost,
                                    hipMemcpyDeviceToDevice, hipMemcpyDeviceToDeviceNoCU};
        HIP_TRY(hipMemcpyAsync(dst, src, (size_t)bytes, k[kind], (hipStream_t)stream));
        return BGX_OK;
    });
}

int bgx_dma_copy_d2h(void* h_dst, const void* d_src, uint64_t bytes, int device, uint64_t* ticket) {
    return guarded("bgx_dma_copy_d2h", [&]() -> int {
        if (!h_dst || !d_src || !ticket) return fail(BGX_E_ARG, "bgx_dma_copy_d2h: null pointer");
        *ticket = 0;
        if (bytes == 0) return BGX_OK;
        DmaDev* d = nullptr;
        if (int rc = dma_setup(device, &d)) return rc;
        void* dst = nullptr;   // the device-visible address of the page-locked host range
        HIP_TRY(hipHostGetDevicePointer(&dst, h_dst, 0));
        // one engine: splitting a copy over several engines moved no more than one
        // (~53-56 GB/s device -> host for 8-32 MiB; profiles/round3/dma_split/)
        hsa_signal_t sig;
        if (hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS)
            return fail(BGX_E_STATE, "bgx_dma_copy_d2h: hsa_signal_create failed");
        const hsa_status_t st = hsa_amd_memory_async_copy_on_engine(dst, d->cpu, d_src, d->gpu, (size_t)bytes, 0,
                                                                    nullptr, sig, d->engine, true);
        if (st != HSA_STATUS_SUCCESS) {
            hsa_signal_destroy(sig);
            return fail(BGX_E_STATE, "bgx_dma_copy_d2h: hsa_amd_memory_async_copy_on_engine failed (%d)", (int)st);
        }
        *ticket = sig.handle;
        return BGX_OK;
    });
}

int bgx_dma_wait(uint64_t ticket, int timeout_ms) {
    return guarded("bgx_dma_wait", [&]() -> int {
        if (ticket == 0) return BGX_OK;
        hsa_signal_t sig;
        sig.handle = ticket;
        const uint64_t ns = timeout_ms > 0 ? (uint64_t)timeout_ms * 1000000ull : UINT64_MAX;
        // spin for the first 2 ms (a harvest's copy takes ~0.1-1 ms; a blocked
        // wait adds an interrupt's wake-up), then sleep in the wait
        const uint64_t spin_ns = ns < 2000000ull ? ns : 2000000ull;
        hsa_signal_value_t v = hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, spin_ns, HSA_WAIT_STATE_ACTIVE);
        if (v >= 1 && ns > spin_ns)
            v = hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, ns - spin_ns, HSA_WAIT_STATE_BLOCKED);
        // past the timeout the copy is still in flight: the ticket stays valid (a
        // later wait may see it end; its signal is destroyed then) and the caller
        // must keep both buffers alive (bgx/hostgather.py STUCK_COPIES)
        if (v >= 1) return fail(BGX_E_STATE, "bgx_dma_wait: copy not finished after %d ms", timeout_ms);
        hsa_signal_destroy(sig);
        return BGX_OK;
    });
}

int bgx_dma_copy_d2d(void* d_dst, int dst_device, const void* d_src, int src_device, uint64_t bytes,
                     uint64_t* ticket) {
    return guarded("bgx_dma_copy_d2d", [&]() -> int {
        if (!d_dst || !d_src || !ticket) return fail(BGX_E_ARG, "bgx_dma_copy_d2d: null pointer");
        *ticket = 0;
        if (bytes == 0) return BGX_OK;
        DmaDev *s = nullptr, *d = nullptr;
        if (int rc = dma_setup(src_device, &s)) return rc;
        if (int rc = dma_setup(dst_device, &d)) return rc;
        // an SDMA engine of the source GPU that serves this pair (xGMI engines for
        // a peer GPU); none listed (e.g. a copy within one GPU on some drivers):
        // the runtime's own choice
        uint32_t mask = 0;
        const bool eng = hsa_amd_memory_copy_engine_status(d->gpu, s->gpu, &mask) == HSA_STATUS_SUCCESS && mask != 0;
        hsa_signal_t sig;
        if (hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS)
            return fail(BGX_E_STATE, "bgx_dma_copy_d2d: hsa_signal_create failed");
        const hsa_status_t st =
            eng ? hsa_amd_memory_async_copy_on_engine(d_dst, d->gpu, d_src, s->gpu, (size_t)bytes, 0, nullptr, sig,
                                                      (hsa_amd_sdma_engine_id_t)(mask & (~mask + 1u)), true)
                : hsa_amd_memory_async_copy(d_dst, d->gpu, d_src, s->gpu, (size_t)bytes, 0, nullptr, sig);
        if (st != HSA_STATUS_SUCCESS) {
            hsa_signal_destroy(sig);
            return fail(BGX_E_STATE, "bgx_dma_copy_d2d: async copy failed (%d)", (int)st);
        }
        *ticket = sig.handle;
        return BGX_OK;
    });
}

int bgx_ipc_export(const void* d_ptr, uint8_t* handle64, uint64_t* offset) {
    return guarded("bgx_ipc_export", [&]() -> int {
        if (!d_ptr || !handle64 || !offset) return fail(BGX_E_ARG, "bgx_ipc_export: null pointer");
        static_assert(sizeof(hipIpcMemHandle_t) == 64, "64-byte IPC handles");
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        HIP_TRY(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)d_ptr));
        hipIpcMemHandle_t h;
        HIP_TRY(hipIpcGetMemHandle(&h, (void*)base));
        std::memcpy(handle64, &h, 64);
        *offset = (uint64_t)((const char*)d_ptr - (const char*)base);
        return BGX_OK;
    });
}

int bgx_ipc_open(const uint8_t* handle64, uint64_t offset, void** d_ptr) {
    return guarded("bgx_ipc_open", [&]() -> int {
        if (!handle64 || !d_ptr) return fail(BGX_E_ARG, "bgx_ipc_open: null pointer");
        hipIpcMemHandle_t h;
        std::memcpy(&h, handle64, 64);
        void* base = nullptr;
        HIP_TRY(hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess));
        *d_ptr = (char*)base + offset;
        return BGX_OK;
    });
}

int bgx_ipc_close(void* d_ptr, uint64_t offset) {
    return guarded("bgx_ipc_close", [&]() -> int {
        if (!d_ptr) return fail(BGX_E_ARG, "bgx_ipc_close: null pointer");
        HIP_TRY(hipIpcCloseMemHandle((char*)d_ptr - offset));
        return BGX_OK;
    });
}

int bgx_reply_moves(const uint8_t* d_boards, const uint8_t* d_opponent, int n, uint32_t* d_out, int cap,
                    int32_t* d_off, int32_t* d_cnt, void* stream) {
    return guarded("bgx_reply_moves", [&]() -> int {
        if (n < 0 || cap < 0) return fail(BGX_E_ARG, "bgx_reply_moves: n=%d cap=%d", n, cap);
        if (n == 0) return BGX_OK;
        if (!d_boards || !d_opponent || !d_out || !d_off || !d_cnt) return fail(BGX_E_ARG, "bgx_reply_moves: null pointer");
        DeviceScope ds(d_boards);
        HIP_TRY(ds.err);
        hipStream_t s = (hipStream_t)stream;
        {
            Lease L;
            if (int rc = lease_scratch(s, L)) return rc;
            if (int rc = require_domain("bgx_reply_moves", L.sc, d_boards, d_opponent, nullptr, n, s)) return rc;
        }
        uint8_t* mover = nullptr;
        uint32_t *rows = nullptr, *ws = nullptr;
        unsigned* ctr = nullptr;
        int32_t* ovf = nullptr;
        int rc = BGX_OK;
        const int ws_waves = 64, ws_slots = 16384, ovf_cap = 1 << 16;
        if (dalloc(&mover, n) || dalloc(&rows, (size_t)n * 8) || dalloc(&ctr, 8) || dalloc(&ovf, ovf_cap) ||
            dalloc(&ws, (size_t)ws_waves * 5 * ws_slots))
            rc = BGX_E_HIP;
        if (!rc) {
            std::vector<uint8_t> ho(n), hm(n);
            if (hipMemcpy(ho.data(), d_opponent, n, hipMemcpyDeviceToHost) != hipSuccess) rc = BGX_E_HIP;
            for (int i = 0; i < n; ++i) hm[i] = (uint8_t)(1 - (ho[i] & 1));   // the candidate's mover
            if (!rc && hipMemcpy(mover, hm.data(), n, hipMemcpyHostToDevice) != hipSuccess) rc = BGX_E_HIP;
        }
        if (!rc && hipMemsetAsync(ctr, 0, 32, s) != hipSuccess) rc = BGX_E_HIP;
        if (!rc && bgx_launch_pack(d_boards, mover, n, rows, s) != hipSuccess) rc = BGX_E_HIP;
        if (!rc) {
            bgx::MovegenArgs b{};
            b.n_jobs = n * 21;
            b.in_mode = bgx::IN_TWOPLY;
            b.in_packed = rows;
            b.out_mode = bgx::OUT_PACKED_FLAT;
            b.out_packed = d_out;
            b.flat_count = ctr;
            b.flat_cap = cap;
            b.flat_chunk = 256;
            b.job_off = d_off;
            b.job_cnt = d_cnt;
            b.ovf_count = ctr + 2;
            b.ovf_list = ovf;
            b.ovf_cap = ovf_cap;
            b.ws_global = ws;
            b.ws_waves = ws_waves;
            b.ws_slots = ws_slots;
            b.ws_words_per_wave = (size_t)5 * ws_slots;
            b.err_flags = ctr + 3;
            if (bgx_launch_movegen(&b, s) != hipSuccess) rc = BGX_E_HIP;
        }
        unsigned flags = 0;
        if (!rc && (hipStreamSynchronize(s) != hipSuccess || hipMemcpy(&flags, ctr + 3, 4, hipMemcpyDeviceToHost) != hipSuccess))
            rc = BGX_E_HIP;
        void* ps[] = {mover, rows, ctr, ovf, ws};
        for (void* p : ps) hipFree(p);
        if (rc) return fail(rc, "bgx_reply_moves: HIP failure");
        if (flags) return fail(BGX_E_CAPACITY, "bgx_reply_moves: overflow flags 0x%x", flags);
        return BGX_OK;
    });
}

int bgx_pack(const uint8_t* d_boards, const uint8_t* d_player, int n, uint32_t* d_packed, void* stream) {
    return guarded("bgx_pack", [&]() -> int {
        if (n < 0) return fail(BGX_E_ARG, "bgx_pack: n=%d", n);
        HIP_TRY(bgx_launch_pack(d_boards, d_player, n, d_packed, (hipStream_t)stream));
        return BGX_OK;
    });
}

int bgx_unpack(const uint32_t* d_packed, int n, uint8_t* d_boards, void* stream) {
    return guarded("bgx_unpack", [&]() -> int {
        if (n < 0) return fail(BGX_E_ARG, "bgx_unpack: n=%d", n);
        HIP_TRY(bgx_launch_unpack(d_packed, n, d_boards, (hipStream_t)stream));
        return BGX_OK;
    });
}

int bgx_net_create(const float* h_W1, const float* h_b1, const float* h_w2, const float* h_b2,
                   bgx_net** out) {
    return guarded("bgx_net_create", [&]() -> int {
        if (!h_W1 || !h_b1 || !h_w2 || !h_b2 || !out) return fail(BGX_E_ARG, "bgx_net_create: null pointer");
        bgx_net* n = new bgx_net();
        if (dalloc(&n->W1, 128 * 198) || dalloc(&n->b1, 128) || dalloc(&n->w2, 128) ||
            dalloc(&n->wfrag, NFRAG) || dalloc(&n->rowc, 128 * 4)) {
            bgx_net_destroy(n);
            return BGX_E_HIP;
        }
        int rc = net_upload(n, h_W1, h_b1, h_w2, h_b2);
        if (rc) {
            bgx_net_destroy(n);
            return rc;
        }
        *out = n;
        return BGX_OK;
    });
}

int bgx_net_destroy(bgx_net* n) {
    return guarded("bgx_net_destroy", [&]() -> int {
        if (!n) return BGX_OK;
        hipFree(n->W1);
        hipFree(n->b1);
        hipFree(n->w2);
        hipFree(n->wfrag);
        hipFree(n->rowc);
        delete n;
        return BGX_OK;
    });
}

int bgx_value(const bgx_net* net, const float* d_x, int n, float* d_out, void* stream) {
    return guarded("bgx_value", [&]() -> int {
        if (!net || n < 0) return fail(BGX_E_ARG, "bgx_value: bad arguments");
        if (n == 0) return BGX_OK;
        HIP_TRY(bgx_launch_value_f32(d_x, n, net->W1, net->b1, net->w2, net->b2, d_out, (hipStream_t)stream));
        return BGX_OK;
    });
}

int bgx_value_boards(const bgx_net* cnet, const uint8_t* d_boards, const uint8_t* d_player, int n,
                     float* d_out, void* stream) {
    return guarded("bgx_value_boards", [&]() -> int {
        bgx_net* net = const_cast<bgx_net*>(cnet);
        if (!net || n < 0) return fail(BGX_E_ARG, "bgx_value_boards: bad arguments");
        if (n == 0) return BGX_OK;
        if (!d_boards || !d_player || !d_out) return fail(BGX_E_ARG, "bgx_value_boards: null pointer");
        DeviceScope ds(d_boards);
        HIP_TRY(ds.err);
        hipStream_t s = (hipStream_t)stream;
        Lease L;
        if (int rc = lease_scratch(s, L)) return rc;
        if (int rc = require_domain("bgx_value_boards", L.sc, d_boards, d_player, nullptr, n, s)) return rc;
        if (L.sc->packed_n < (size_t)n) {   // the lease's last user has finished (lease_scratch)
            hipFree(L.sc->packed);
            L.sc->packed = nullptr;
            L.sc->packed_n = 0;
            if (dalloc(&L.sc->packed, (size_t)n * 8)) return BGX_E_HIP;
            L.sc->packed_n = (size_t)n;
        }
        HIP_TRY(bgx_launch_pack(d_boards, d_player, n, L.sc->packed, s));
        bgx::MlpArgs m{};
        m.rows = L.sc->packed;
        m.n_rows = n;
        m.out = d_out;
        m.wfrag = net->wfrag;
        m.rowc = net->rowc;
        m.b2 = net->b2;
        m.feat_scale = net->feat_scale;
        HIP_TRY(bgx_launch_mlp(&m, s));
        return BGX_OK;
    });
}

int bgx_two_ply(const bgx_net* net, const uint8_t* d_boards, const uint8_t* d_opponent, int n,
                double* d_out, void* stream) {
    return guarded("bgx_two_ply", [&]() -> int {
        return bgx_two_ply_sampled(net, d_boards, d_opponent, n, 0, 0, d_out, stream);
    });
}

// BGX_REPLY_DELTA=1: the 2-ply reply values by difference from their roots
// (mlp_kernel_delta, bgx_mlp.hip) instead of in full (mlp_kernel_il, the
// default). Measured and not kept: 33 % fewer MFMAs but
// twice the VALU and 27x the SALU instructions per tile, 0.95 vs 0.69 ms per
// K = 4 reply launch. Read when an engine is created / per stateless call, so
// tests can cross-check both forms in one process.
static bool reply_delta() {
    const char* v = getenv("BGX_REPLY_DELTA");
    return v && atoi(v) != 0;
}

int bgx_two_ply_sampled(const bgx_net* net, const uint8_t* d_boards, const uint8_t* d_opponent, int n,
                        int sample_k, uint64_t seed, double* d_out, void* stream) {
    return guarded("bgx_two_ply_sampled", [&]() -> int {
        if (!net || n < 0) return fail(BGX_E_ARG, "bgx_two_ply: bad arguments");
        if (sample_k != 0 && (sample_k < 5 || sample_k > 1024))
            return fail(BGX_E_ARG, "bgx_two_ply_sampled: sample_k=%d (0 = exact, 5..1024)", sample_k);
        if (n == 0) return BGX_OK;
        if (!d_boards || !d_opponent || !d_out) return fail(BGX_E_ARG, "bgx_two_ply: null pointer");
        DeviceScope ds(d_boards);
        HIP_TRY(ds.err);
        hipStream_t s = (hipStream_t)stream;
        {
            Lease L;
            if (int rc = lease_scratch(s, L)) return rc;
            if (int rc = require_domain("bgx_two_ply", L.sc, d_boards, d_opponent, nullptr, n, s)) return rc;
        }
        const int jobs = n * 21;
        const int cap = jobs * 768;   // >= any reply count per (board, roll)
        uint8_t* mover = nullptr;
        uint32_t *rows = nullptr, *reply = nullptr, *ws = nullptr;
        unsigned* ctr = nullptr;
        int32_t *off = nullptr, *cnt = nullptr, *ovf = nullptr;
        float *V = nullptr, *jv = nullptr;
        int rc = BGX_OK;
        const int ws_waves = 64, ws_slots = 16384, ovf_cap = 1 << 16;
        if (dalloc(&mover, n) || dalloc(&rows, (size_t)n * 8) || dalloc(&reply, (size_t)cap * 8) ||
            dalloc(&ctr, 8) || dalloc(&off, jobs) || dalloc(&cnt, jobs) || dalloc(&V, cap) || dalloc(&jv, jobs) ||
            dalloc(&ovf, ovf_cap) || dalloc(&ws, (size_t)ws_waves * 5 * ws_slots)) {
            rc = BGX_E_HIP;
        }
        std::vector<uint8_t> hm;
        if (!rc) {
            // the candidate board's indicator = the player who just moved = 1 - opponent
            std::vector<uint8_t> ho(n);
            if (hipMemcpy(ho.data(), d_opponent, n, hipMemcpyDeviceToHost) != hipSuccess) rc = BGX_E_HIP;
            hm.resize(n);
            for (int i = 0; i < n; ++i) hm[i] = (uint8_t)(1 - (ho[i] & 1));
        }
        if (!rc && hipMemcpy(mover, hm.data(), n, hipMemcpyHostToDevice) != hipSuccess) rc = BGX_E_HIP;
        if (!rc && hipMemsetAsync(ctr, 0, 32, s) != hipSuccess) rc = BGX_E_HIP;
        if (!rc && bgx_launch_pack(d_boards, mover, n, rows, s) != hipSuccess) rc = BGX_E_HIP;
        if (!rc) {
            bgx::MovegenArgs b{};
            b.n_jobs = jobs;
            b.in_mode = bgx::IN_TWOPLY;
            b.in_packed = rows;
            b.in_rows = nullptr;
            b.in_row_base = 0;
            b.out_mode = bgx::OUT_PACKED_FLAT;
            b.out_packed = reply;
            b.flat_count = ctr;
            b.flat_cap = cap;
            b.flat_chunk = 256;
            b.job_off = off;
            b.job_cnt = cnt;
            b.ovf_count = ctr + 2;
            b.ovf_list = ovf;
            b.ovf_cap = ovf_cap;
            b.ws_global = ws;
            b.ws_waves = ws_waves;
            b.ws_slots = ws_slots;
            b.ws_words_per_wave = (size_t)5 * ws_slots;
            b.err_flags = ctr + 3;
            if (bgx_launch_movegen(&b, s) != hipSuccess) rc = BGX_E_HIP;
        }
        float* zt = nullptr;
        if (!rc && reply_delta()) {
            // the roots' hidden accumulators (their V goes to the reply buffer's
            // first n slots, overwritten below), for the replies by difference
            if (dalloc(&zt, (size_t)n * 128)) rc = BGX_E_HIP;
            bgx::MlpArgs m{};
            m.rows = rows;
            m.n_rows = n;
            m.nt = 1;
            m.out = V;
            m.wfrag = net->wfrag;
            m.rowc = net->rowc;
            m.b2 = net->b2;
            m.feat_scale = net->feat_scale;
            m.zout = zt;
            m.z_base = 0;
            if (!rc && bgx_launch_mlp(&m, s) != hipSuccess) rc = BGX_E_HIP;
        }
        if (!rc) {
            bgx::MlpArgs m{};
            m.rows = reply;
            m.n_rows = 0;
            m.n_rows_dev = ctr;
            m.n_max = cap;
            m.nt = 2;
            m.out = V;
            m.wfrag = net->wfrag;
            m.rowc = net->rowc;
            m.b2 = net->b2;
            m.feat_scale = net->feat_scale;
            if (zt) {
                m.zt = zt;
                m.root_rows = rows;
                m.root_sel = nullptr;
                m.root_base = 0;
                m.n_roots = n;
                m.n_slots = n;
            }
            if (bgx_launch_mlp(&m, s) != hipSuccess) rc = BGX_E_HIP;
        }
        if (!rc && bgx_launch_top5(V, off, cnt, jobs, nullptr, 0, jobs, jv, sample_k, seed, nullptr, nullptr, s) != hipSuccess)
            rc = BGX_E_HIP;
        if (!rc && bgx_launch_two_ply_reduce(jv, n, d_out, s) != hipSuccess) rc = BGX_E_HIP;
        unsigned flags = 0;
        if (!rc && (hipStreamSynchronize(s) != hipSuccess || hipMemcpy(&flags, ctr + 3, 4, hipMemcpyDeviceToHost) != hipSuccess))
            rc = BGX_E_HIP;
        void* ps[] = {mover, rows, reply, ctr, off, cnt, V, jv, ovf, ws, zt};
        for (void* p : ps) hipFree(p);
        if (rc) return fail(rc, "bgx_two_ply: HIP failure");
        if (flags) return fail(BGX_E_CAPACITY, "bgx_two_ply: overflow flags 0x%x", flags);
        return BGX_OK;
    });
}

void bgx_config_default(bgx_config* c) {
    std::memset(c, 0, sizeof(*c));
    c->lanes = 4096;
    c->lane_base = 0;
    c->seed = 0;
    c->ply = 1;
    c->k_top = 4;
    c->alpha = 1.0f;
    c->beta = 0.9f;
    c->max_steps = 300;
    c->max_legal = 500;
    c->ring = 1024;
    c->ep_cap = 0;   // 0 = derived from lanes
    c->cand_per_lane = 256;
    c->reply_per_lane = 0;   // 0 = derived from k_top
    c->fused = 1;
}

int bgx_engine_destroy(bgx_engine* e) {
    return guarded("bgx_engine_destroy", [&]() -> int {
        if (!e) return BGX_OK;
        hipSetDevice(e->device);
        hipDeviceSynchronize();
        if (e->fprof) {   // development report (BGX_FUSED_PROF): per workgroup-step averages, wall clock 100 MHz
            std::vector<unsigned long long> p((size_t)1024 * PROF_W);
            if (hipMemcpy(p.data(), e->fprof, p.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
                double s[32] = {0};
                for (int b = 0; b < 1024; ++b)
                    for (int k = 0; k < 23; ++k) s[k] += (double)p[(size_t)b * PROF_W + k];
                const double n = s[5] > 0 ? s[5] : 1;
                const double nws = s[18] > 0 ? s[18] : 1;   // wave-steps
                // (the pipelined kernel: each step is tier 2 + the row prefix, then one item
                // queue of MLP tiles, choice pairs and the next step's tier-1 jobs)
                fprintf(stderr, "[bgx fused prof] us per workgroup step: tier2 + prefix %.2f, queue %.2f, end barrier %.2f "
                        "(%.0f workgroup steps)\n", s[1] / n / 100, s[3] / n / 100, s[4] / n / 100, n);
                fprintf(stderr, "[bgx fused prof] wave-us per workgroup step in items: MLP tiles %.2f, choice pairs %.2f, "
                        "tier-1 jobs %.2f (%.2f per wave-step of %d waves)\n", s[8] / n / 100, s[10] / n / 100,
                        (s[14] + s[16]) / n / 100, (s[8] + s[10] + s[14] + s[16]) / nws / 100, (int)(nws / n + 0.5));
                {
                    double c[3] = {0, 0, 0};
                    for (int b = 0; b < 1024; ++b)
                        for (int k = 0; k < 3; ++k) c[k] += (double)p[(size_t)b * PROF_W + 29 + k];
                    fprintf(stderr, "[bgx fused prof] choice per wave-step: state + Philox refill %.2f, pick %.2f, "
                            "env step %.2f us\n", c[0] / nws / 100, c[1] / nws / 100, c[2] / nws / 100);
                }
                {
                    double c[3] = {0, 0, 0};
                    for (int b = 0; b < 1024; ++b) {
                        c[0] += (double)p[(size_t)b * PROF_W + 6];
                        c[1] += (double)p[(size_t)b * PROF_W + 22];
                        c[2] += (double)p[(size_t)b * PROF_W + 23];
                    }
                    fprintf(stderr, "[bgx fused prof] MLP tiles per workgroup step: rows + k mask %.2f, MFMA chain issue %.2f, "
                            "drain + epilogue %.2f wave-us\n", c[0] / n / 100, c[1] / n / 100, c[2] / n / 100);
                }
                {   // step durations by index within a launch (every launch, every workgroup)
                    double st[24] = {0}, cn[24] = {0}, late = 0, nlate = 0;
                    for (int b = 0; b < 1024; ++b) {
                        for (int k = 0; k < 24; ++k) {
                            st[k] += (double)p[(size_t)b * PROF_W + 32 + k];
                            cn[k] += (double)p[(size_t)b * PROF_W + 64 + k];
                        }
                        late += (double)p[(size_t)b * PROF_W + 56];
                        nlate += (double)p[(size_t)b * PROF_W + 57];
                    }
                    fprintf(stderr, "[bgx fused prof] step us by index in the launch (workgroup-steps):");
                    for (int k = 0; k < 24; ++k) fprintf(stderr, " %.2f (%.0f)", cn[k] > 0 ? st[k] / cn[k] / 100 : 0.0, cn[k]);
                    fprintf(stderr, "; later steps %.2f (%.0f)\n", nlate > 0 ? late / nlate / 100 : 0.0, nlate);
                }
                fprintf(stderr, "[bgx fused prof] tier-2 jobs %.0f (%.0f reached tier 3), %.1f us each\n", s[12], s[13],
                        s[11] / (s[12] > 0 ? s[12] : 1) / 100);
                fprintf(stderr, "[bgx fused prof] tier-1 job: doubles %.2f us (%.0f jobs), non-doubles %.2f us (%.0f jobs)\n",
                        s[14] / (s[15] > 0 ? s[15] : 1) / 100, s[15], s[16] / (s[17] > 0 ? s[17] : 1) / 100, s[17]);
                // the last launch, per workgroup: duration spread, dispatch skew, and the
                // rows / tier-2 jobs of the slowest vs the median workgroup
                std::vector<std::pair<double, int>> dur;
                unsigned long long b_min = ~0ull, b_max = 0, e_max = 0;
                for (int b = 0; b < 1024; ++b) {
                    const unsigned long long* q = &p[(size_t)b * PROF_W];
                    if (q[25] <= q[24]) continue;
                    dur.push_back({(double)(q[25] - q[24]) / 100.0, b});
                    b_min = q[24] < b_min ? q[24] : b_min;
                    b_max = q[24] > b_max ? q[24] : b_max;
                    e_max = q[25] > e_max ? q[25] : e_max;
                }
                if (const char* path = getenv("BGX_FUSED_PROF_DUMP")) {
                    // the last launch per workgroup: begin / end clocks (100 MHz),
                    // loop start / end, rows, tier-2 jobs, lane-steps
                    if (FILE* fp = fopen(path, "w")) {
                        fprintf(fp, "wg,begin,end,loop0,loop1,rows,tier2,lane_steps\n");
                        for (int b = 0; b < 1024; ++b) {
                            const unsigned long long* q = &p[(size_t)b * PROF_W];
                            if (q[25] <= q[24]) continue;
                            fprintf(fp, "%d,%llu,%llu,%llu,%llu,%llu,%llu,%llu\n", b, q[24], q[25], q[19], q[20], q[26],
                                    q[27], q[28]);
                        }
                        fclose(fp);
                    }
                }
                if (!dur.empty()) {
                    std::sort(dur.begin(), dur.end());
                    double mean = 0;
                    for (auto& d : dur) mean += d.first;
                    mean /= (double)dur.size();
                    const size_t nd = dur.size();
                    const unsigned long long* qm = &p[(size_t)dur[nd / 2].second * 32];
                    const unsigned long long* qx = &p[(size_t)dur[nd - 1].second * 32];
                    fprintf(stderr, "[bgx fused prof] last launch, %zu workgroups: duration us min %.1f p50 %.1f mean %.1f "
                            "p90 %.1f max %.1f; begin skew %.1f us, span %.1f us; lane-steps %llu; rows / tier-2 jobs: "
                            "median workgroup %llu / %llu, slowest %llu / %llu\n",
                            nd, dur[0].first, dur[nd / 2].first, mean, dur[(nd * 9) / 10].first, dur[nd - 1].first,
                            (double)(b_max - b_min) / 100.0, (double)(e_max - b_min) / 100.0, qx[28], qm[26], qm[27],
                            qx[26], qx[27]);
                    // launch shape (median workgroup): prologue (W fragments, LUT, lane
                    // state), the step loop, epilogue (lane state back); shader clock
                    // over the workgroup's span (s_memtime cycles / 100 MHz wall clock)
                    std::vector<double> pro, loop, epi, mhz;
                    for (auto& d : dur) {
                        const unsigned long long* q = &p[(size_t)d.second * 32];
                        if (q[19] < q[24] || q[20] < q[19] || q[25] < q[20]) continue;
                        pro.push_back((double)(q[19] - q[24]) / 100.0);
                        loop.push_back((double)(q[20] - q[19]) / 100.0);
                        epi.push_back((double)(q[25] - q[20]) / 100.0);
                        mhz.push_back((double)q[21] / ((double)(q[25] - q[24]) / 100.0));
                    }
                    if (!pro.empty()) {
                        auto med = [](std::vector<double>& v) {
                            std::sort(v.begin(), v.end());
                            return v[v.size() / 2];
                        };
                        fprintf(stderr, "[bgx fused prof] last launch shape (median workgroup): prologue %.1f us, step loop "
                                "%.1f us, epilogue %.1f us; shader clock %.0f MHz\n", med(pro), med(loop), med(epi),
                                med(mhz));
                    }
                }
            }
            hipFree(e->fprof);
        }
        void* ps[] = {e->rows, e->V, e->cand_off, e->cand_cnt, e->ctr, e->stats, e->sel, e->sel_rows, e->reply_rows,
                      e->reply_V, e->job_off, e->job_cnt, e->job_val, e->zt, e->zv, e->ovf_list, e->ws, e->out_records[0],
                      e->out_records[1], e->out_records[2], e->out_headers[0], e->out_headers[1], e->out_headers[2],
                      e->d_offs[0], e->d_offs[1], e->d_offs[2], e->d_info[2], e->fh_ctr, e->d.hring, e->d.hepi,
                      e->d_info[0], e->d_info[1], e->fcand, e->fvbuf, e->ft1cnt, e->d.player, e->d.dice, e->d.step, e->d.flags, e->d.epi, e->d.rng,
                      e->d.rec_count, e->d.ep_first, e->d.harv, e->d.ring, e->d.ep_list, e->dice_tab};
        for (void* p : ps) hipFree(p);
        for (hipEvent_t ev : e->ev) hipEventDestroy(ev);
        if (e->gexec) hipGraphExecDestroy(e->gexec);
        if (e->hev) hipEventDestroy(e->hev);
        for (hipEvent_t ev : e->hdone)
            if (ev) hipEventDestroy(ev);
        if (e->h_info) hipHostFree(e->h_info);
        if (e->cap) hipStreamDestroy(e->cap);
        bgx_net_destroy(e->net);
        delete e;
        return BGX_OK;
    });
}

// Rows per reply-launch reservation unit (MovegenArgs::flat_chunk): 512 by
// default, BGX_FLAT_CHUNK in [64, 1024] for A/B runs (the engine's reply_cap
// slack is sized from it, so it is bounded above too).
static int reply_flat_chunk() {
    static const int chunk = [] {
        const char* v = getenv("BGX_FLAT_CHUNK");
        const int c = v ? atoi(v) : 512;
        return c < 64 ? 512 : (c > 1024 ? 1024 : c);
    }();
    return chunk;
}

int bgx_engine_create(int device, const bgx_config* cfg, bgx_engine** out) {
    return guarded("bgx_engine_create", [&]() -> int {
        if (!cfg || !out) return fail(BGX_E_ARG, "bgx_engine_create: null pointer");
        if (cfg->lanes <= 0 || cfg->lanes > (1 << 24)) return fail(BGX_E_ARG, "lanes=%d", cfg->lanes);
        if (cfg->ply != 1 && cfg->ply != 2) return fail(BGX_E_ARG, "ply=%d (1 or 2)", cfg->ply);
        if (cfg->ply == 2 && cfg->k_top != 4 && cfg->k_top != 0)
            return fail(BGX_E_ARG, "k_top=%d (4 = reference, 0 = all)", cfg->k_top);
        if (cfg->reply_sample != 0 && (cfg->reply_sample < 5 || cfg->reply_sample > 1024))
            return fail(BGX_E_ARG, "reply_sample=%d (0 = exact, 5..1024; the reference samples 50)", cfg->reply_sample);
        if (cfg->max_steps <= 0 || cfg->max_legal <= 0) return fail(BGX_E_ARG, "max_steps/max_legal");
        if (cfg->ring < cfg->max_steps + 1 || cfg->ring > (1 << 16))
            return fail(BGX_E_ARG, "ring=%d (max_steps+1 .. 65536)", cfg->ring);
        // the select kernel keeps a lane's scores in a 512-entry LDS row; the fused
        // 1-ply kernel keeps its candidates in per-lane slots of max_legal
        const bool fused_cfg = cfg->fused != 0 && cfg->ply == 1;
        if (cfg->max_legal > (fused_cfg ? 2048 : 512))
            return fail(BGX_E_ARG, "max_legal=%d > %d (%s engine)", cfg->max_legal, fused_cfg ? 2048 : 512,
                        fused_cfg ? "fused" : "phased");
        if (cfg->max_steps > 511) return fail(BGX_E_ARG, "max_steps=%d > 511 (record step field)", cfg->max_steps);
        HIP_TRY(hipSetDevice(device));
        bgx_engine* e = new bgx_engine();
        e->device = device;
        if (const char* g = getenv("BGX_GRAPH")) e->use_graph = atoi(g) != 0;
        if (const char* v = getenv("BGX_MG_TEST_TIER")) e->force_tier = atoi(v);
        e->prof_enabled = getenv("BGX_FUSED_PROF") != nullptr;
        if (const char* v = getenv("BGX_FUSED_LANES")) e->fused_fl = atoi(v);
        e->cfg = *cfg;
        // ring slots: a power of two (slot = record counter & (R - 1) stays exact
        // when the 32-bit counter wraps)
        int ring = 1;
        while (ring < cfg->ring) ring <<= 1;
        e->cfg.ring = ring;
        const int L = cfg->lanes;
        e->cand_cap = L * (cfg->cand_per_lane > 0 ? cfg->cand_per_lane : 256);
        // finished episodes between two harvests: at most (steps per harvest) /
        // (shortest game) + 1 per lane. A game takes >= 7 turns of the winner
        // (167 pips, at most 24 per turn) and >= 6 of the loser: >= 13 env steps.
        constexpr int kMinGameSteps = 13;
        const long long ep_need = (long long)L * ((ring - cfg->max_steps) / kMinGameSteps + 1) + 1024;
        const int ep_cap = cfg->ep_cap > 0 ? cfg->ep_cap : (int)(ep_need < (1 << 30) ? ep_need : (1 << 30));
        int rc = BGX_OK;
        bgx::EngineDev& d = e->d;
    #define ALLOC(p, n) \
        if (!rc) rc = dalloc(&(p), (size_t)(n))
        ALLOC(e->rows, (size_t)(L + e->cand_cap) * 8);
        ALLOC(e->V, (size_t)(L + e->cand_cap));
        ALLOC(e->cand_off, L);
        ALLOC(e->cand_cnt, L);
        ALLOC(e->ctr, 16);
        ALLOC(e->stats, kStatWords);
        ALLOC(d.player, L);
        ALLOC(d.dice, 2 * L);
        ALLOC(d.step, L);
        ALLOC(d.flags, L);
        ALLOC(d.epi, L);
        ALLOC(d.rng, L);
        ALLOC(d.rec_count, L);
        ALLOC(d.ep_first, L);
        ALLOC(d.harv, L);
        ALLOC(d.ring, (size_t)L * ring * bgx::REC_WORDS);
        ALLOC(d.ep_list, (size_t)ep_cap * bgx::EP_WORDS);
        for (int b = 0; b < bgx_engine::NHB; ++b) {
            ALLOC(e->out_records[b], (size_t)L * ring * bgx::REC_WORDS);
            ALLOC(e->out_headers[b], (size_t)ep_cap * bgx::EP_WORDS);
            ALLOC(e->d_offs[b], (size_t)ep_cap + 1);
            ALLOC(e->d_info[b], 4);
            if (!rc && hipEventCreateWithFlags(&e->hdone[b], hipEventDisableTiming) != hipSuccess)
                rc = fail(BGX_E_HIP, "hipEventCreate failed");
        }
        if (!rc && (hipHostMalloc((void**)&e->h_info, 4 * bgx_engine::NHB * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent) !=
                        hipSuccess ||
                    hipHostGetDevicePointer((void**)&e->h_info_dev, e->h_info, 0) != hipSuccess))
            rc = fail(BGX_E_HIP, "hipHostMalloc (mapped) failed");
        e->ovf_cap = 1 << 16;
        e->ws_waves = 512;   // one global-memory fallback slice per tier-2 block / fused workgroup (<= 2 per CU)
        e->ws_slots = 16384;
        ALLOC(e->ovf_list, e->ovf_cap);
        ALLOC(e->ws, (size_t)e->ws_waves * 5 * e->ws_slots);
        e->fused = fused_cfg;
        if (e->fused) {
            e->fcap = cfg->max_legal;
            ALLOC(e->fcand, (size_t)L * e->fcap * 8);
            ALLOC(e->fvbuf, (size_t)L * (e->fcap + 1));
            ALLOC(e->ft1cnt, L);
            // per-lane episode headers for the in-kernel harvest: at most
            // (ring - max_steps) / 13 + 1 episodes finish between two harvests
            int hr = 1;
            while (hr < (ring - cfg->max_steps) / kMinGameSteps + 2) hr <<= 1;
            d.HR = hr;
            ALLOC(d.hring, (size_t)L * hr * bgx::EP_WORDS);
            ALLOC(d.hepi, L);
            ALLOC(e->fh_ctr, 3 * bgx_engine::NHB + 1);   // reservations, done, flags, commits
        }
        if (cfg->ply == 2) {
            e->jobs_cap = cfg->k_top == 4 ? L * 4 * 21 : e->cand_cap * 21;
            const int per_lane = cfg->reply_per_lane > 0 ? cfg->reply_per_lane : (cfg->k_top == 4 ? 4096 : 16384);
            int n_cu = 256;
            if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) n_cu = 256;
            // + slack for the rows reserved but left unwritten: the reply launch
            // runs two workgroups per CU (bgx_launch_movegen), each ending with at
            // most one workgroup chunk (<= 8 x flat_chunk rows) and its waves'
            // kept remainders (tails of replaced chunks, each smaller than the
            // request that replaced it); two chunks' worth per workgroup covers
            // both (measured gap rows: 2-3 % of a K = 4 step's rows, DESIGN.md
            // section 4). Running out is flagged (BGX_E_CAPACITY), not silent.
            e->reply_cap = L * per_lane + n_cu * 2 * 2 * 8 * reply_flat_chunk();
            ALLOC(e->sel, 4 * L);
            ALLOC(e->sel_rows, (size_t)4 * L * 8);
            ALLOC(e->reply_rows, (size_t)e->reply_cap * 8);
            ALLOC(e->reply_V, e->reply_cap);
            ALLOC(e->job_off, e->jobs_cap);
            ALLOC(e->job_cnt, e->jobs_cap);
            ALLOC(e->job_val, e->jobs_cap);
            if (reply_delta()) {
                ALLOC(e->zt, (size_t)(cfg->k_top == 4 ? 4 * L : e->cand_cap) * 128);
                if (cfg->k_top == 4) ALLOC(e->zv, 4 * L);
            }
        }
    #undef ALLOC
        if (rc) {
            bgx_engine_destroy(e);
            return rc;
        }
        if (hipMemset(e->ctr, 0, 64) != hipSuccess || hipMemset(e->stats, 0, kStatWords * sizeof(unsigned long long)) != hipSuccess ||
            (e->fh_ctr && hipMemset(e->fh_ctr, 0, (3 * bgx_engine::NHB + 1) * sizeof(unsigned long long)) != hipSuccess)) {
            bgx_engine_destroy(e);
            return fail(BGX_E_HIP, "hipMemset failed");
        }
        d.L = L;
        d.lane_base = cfg->lane_base;
        d.seed = cfg->seed;
        d.temperature = 1.5f;
        d.max_steps = cfg->max_steps;
        d.max_legal = cfg->max_legal;
        d.ply = cfg->ply;
        d.k_top = cfg->k_top;
        d.alpha = cfg->alpha;
        d.greedy = cfg->greedy != 0;
        d.beta = cfg->beta;
        d.rows = e->rows;
        d.cand_cap = e->cand_cap;
        d.R = ring;
        d.dice_tab = nullptr;
        d.dice_len = 0;
        d.ep_count = e->ctr + C_EP;
        d.ep_cap = ep_cap;
        d.cand_off = e->cand_off;
        d.cand_cnt = e->cand_cnt;
        d.V = e->V;
        d.sel = e->sel;
        d.sel_rows = e->sel_rows;
        d.job_val = e->job_val;
        d.flat_count = e->ctr + C_FLAT;
        d.reply_count = e->ctr + C_REPLY;
        d.ovf_count = e->ctr + C_OVF;
        d.ovf_count2 = e->ctr + C_OVF2;
        d.n_jobs2 = cfg->k_top == 4 ? L * 4 * 21 : 0;
        d.stats = e->stats;
        d.err_flags = e->ctr + C_ERR;
        if (bgx_launch_engine_reset(&d, nullptr) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
            bgx_engine_destroy(e);
            return fail(BGX_E_HIP, "engine reset failed");
        }
        *out = e;
        return BGX_OK;
    });
}

int bgx_engine_set_dice(bgx_engine* e, const uint8_t* h_dice, int per_lane) {
    return guarded("bgx_engine_set_dice", [&]() -> int {
        if (!e || !h_dice || per_lane < 2) return fail(BGX_E_ARG, "bgx_engine_set_dice: bad arguments");
        if (!e->cfg.greedy) return fail(BGX_E_STATE, "bgx_engine_set_dice: scripted dice need greedy play");
        const size_t n = (size_t)e->cfg.lanes * (size_t)per_lane;
        for (size_t k = 0; k < n; ++k)
            if (h_dice[k] < 1 || h_dice[k] > 6) return fail(BGX_E_ARG, "bgx_engine_set_dice: die %d at %zu", h_dice[k], k);
        HIP_TRY(hipSetDevice(e->device));
        if (e->last) HIP_TRY(hipStreamSynchronize(e->last));
        hipFree(e->dice_tab);
        e->dice_tab = nullptr;
        if (dalloc(&e->dice_tab, n)) return BGX_E_HIP;
        HIP_TRY(hipMemcpy(e->dice_tab, h_dice, n, hipMemcpyHostToDevice));
        e->d.dice_tab = e->dice_tab;
        e->d.dice_len = per_lane;
        if (e->gexec) {
            HIP_TRY(hipGraphExecDestroy(e->gexec));
            e->gexec = nullptr;
        }
        // every lane restarts from BackgammonEnv.reset with its scripted dice
        HIP_TRY(hipMemset(e->ctr, 0, 64));
        HIP_TRY(bgx_launch_engine_reset(&e->d, nullptr));
        e->t1_ready = false;   // the fused launch's carried expansion belongs to the old positions
        HIP_TRY(hipDeviceSynchronize());
        return check_flags(e);
    });
}

int bgx_set_weights(bgx_engine* e, const float* h_W1, const float* h_b1, const float* h_w2,
                    const float* h_b2, float temperature, uint64_t version) {
    return guarded("bgx_set_weights", [&]() -> int {
        (void)version;
        if (!e) return fail(BGX_E_ARG, "bgx_set_weights: null engine");
        if (!(temperature > 0.0f)) return fail(BGX_E_ARG, "temperature=%g", (double)temperature);
        HIP_TRY(hipSetDevice(e->device));
        if (e->last) HIP_TRY(hipStreamSynchronize(e->last));
        if (!e->net) {
            int rc = bgx_net_create(h_W1, h_b1, h_w2, h_b2, &e->net);
            if (rc) return rc;
        } else {
            int rc = net_upload(e->net, h_W1, h_b1, h_w2, h_b2);
            if (rc) return rc;
        }
        if (e->gexec && e->d.temperature != temperature) {
            HIP_TRY(hipGraphExecDestroy(e->gexec));
            e->gexec = nullptr;
        }
        e->d.temperature = temperature;
        return BGX_OK;
    });
}

static void mg_common(bgx_engine* e, bgx::MovegenArgs& a) {
    a.ovf_count = e->ctr + C_OVF;
    a.ovf_zeroed = 1;   // the per-step memset covers it
    a.ovf_list = e->ovf_list;
    a.ovf_cap = e->ovf_cap;
    a.ws_global = e->ws;
    a.ws_waves = e->ws_waves;
    a.ws_slots = e->ws_slots;
    a.ws_words_per_wave = (size_t)5 * e->ws_slots;
    a.err_flags = e->ctr + C_ERR;
}

static int timed(bgx_engine* e, int kind, hipStream_t s, bool start) {
    if (!e->timing) return BGX_OK;
    hipEvent_t ev;
    HIP_TRY(hipEventCreate(&ev));
    HIP_TRY(hipEventRecord(ev, s));
    e->ev.push_back(ev);
    e->ev_kind.push_back(start ? kind : -1);
    return BGX_OK;
}

// the per-step launch sequence (captured into a graph by bgx_step)
static int enqueue_steps(bgx_engine* e, int n_steps, hipStream_t s) {
    const int L = e->cfg.lanes;
    for (int it = 0; it < n_steps; ++it) {
        // the per-step counters (flat, reply, ovf, ovf2) are zero here: engine
        // create zeroes them and every step's last kernel resets them
        bgx::MovegenArgs a{};
        a.n_jobs = L;
        a.in_mode = bgx::IN_PACKED;
        a.in_packed = e->rows;
        a.in_player = e->d.player;
        a.in_dice = e->d.dice;
        a.out_mode = bgx::OUT_PACKED_FLAT;
        a.out_packed = e->rows + (size_t)L * 8;
        a.flat_count = e->ctr + C_FLAT;
        a.flat_cap = e->cand_cap;
        a.job_off = e->cand_off;
        a.job_cnt = e->cand_cnt;
        mg_common(e, a);
        if (timed(e, 0, s, true)) return BGX_E_HIP;
        HIP_TRY(bgx_launch_movegen(&a, s));
        if (timed(e, 0, s, false)) return BGX_E_HIP;

        bgx::MlpArgs m{};
        m.rows = e->rows;
        m.n_rows = L;
        m.n_rows_dev = e->ctr + C_FLAT;
        m.n_max = L + e->cand_cap;
        m.out = e->V;
        m.wfrag = e->net->wfrag;
        m.rowc = e->net->rowc;
        m.b2 = e->net->b2;
        m.feat_scale = e->net->feat_scale;
        if (e->zt && e->cfg.k_top != 4) {   // 2-ply K = all: every candidate's accumulators (the reply roots)
            m.zout = e->zt;
            m.z_base = L;
        }
        if (timed(e, 1, s, true)) return BGX_E_HIP;
        HIP_TRY(bgx_launch_mlp(&m, s));
        if (timed(e, 1, s, false)) return BGX_E_HIP;

        if (e->cfg.ply == 2) {
            bgx::MovegenArgs b{};
            b.in_mode = bgx::IN_TWOPLY;
            b.in_packed = e->rows;
            if (e->cfg.k_top == 4) {
                HIP_TRY(bgx_launch_topk(&e->d, s));
                if (e->zt) {   // the chosen rows' accumulators, indexed by reply root slot (4 lane + k)
                    bgx::MlpArgs z{};
                    z.rows = e->sel_rows;
                    z.n_rows = 4 * L;
                    z.nt = 1;
                    z.out = e->zv;
                    z.wfrag = e->net->wfrag;
                    z.rowc = e->net->rowc;
                    z.b2 = e->net->b2;
                    z.feat_scale = e->net->feat_scale;
                    z.zout = e->zt;
                    z.z_base = 0;
                    HIP_TRY(bgx_launch_mlp(&z, s));
                }
                b.n_jobs = L * 4 * 21;
                b.in_packed = e->sel_rows;   // the top-k kernel's copies of the chosen rows
                b.in_rows = nullptr;
                b.in_row_base = 0;
            } else {
                b.n_jobs = 0;
                b.n_jobs_dev = e->ctr + C_FLAT;
                b.jobs_per_dev_unit = 21;
                b.n_jobs_max = e->jobs_cap;
                b.in_rows = nullptr;
                b.in_row_base = L;
            }
            b.out_mode = bgx::OUT_PACKED_FLAT;
            b.out_packed = e->reply_rows;
            b.flat_count = e->ctr + C_REPLY;
            b.flat_cap = e->reply_cap;
            // output-row reservations: the reply launch's workgroups take chunks of
            // up to 8 x flat_chunk rows per global atomic (bgx_movegen.h wg_take),
            // the per-roll pool kernel's waves chunks of up to flat_chunk; a
            // chunk's unwritten tail is gap rows the reply MLP evaluates
            // (bgx_stats.gap_rows)
            b.flat_chunk = reply_flat_chunk();
            b.job_off = e->job_off;
            b.job_cnt = e->job_cnt;
            mg_common(e, b);
            b.ovf_count = e->ctr + C_OVF2;
            if (timed(e, 0, s, true)) return BGX_E_HIP;
            HIP_TRY(bgx_launch_movegen(&b, s));
            if (timed(e, 0, s, false)) return BGX_E_HIP;
            bgx::MlpArgs r{};
            r.rows = e->reply_rows;
            r.n_rows = 0;
            r.n_rows_dev = e->ctr + C_REPLY;
            r.n_max = e->reply_cap;
            r.nt = 2;
            r.out = e->reply_V;
            r.wfrag = e->net->wfrag;
            r.rowc = e->net->rowc;
            r.b2 = e->net->b2;
            r.feat_scale = e->net->feat_scale;
            if (e->zt) {   // replies by difference from their roots (mlp_kernel_delta)
                const bool k4 = e->cfg.k_top == 4;
                r.zt = e->zt;
                r.root_rows = k4 ? e->sel_rows : e->rows;   // K = 4: the top-k kernel's copies, by slot
                r.root_sel = nullptr;
                r.root_base = k4 ? 0 : L;
                r.n_roots = k4 ? 4 * L : e->cand_cap;
                r.n_slots = r.n_roots;
            }
            if (timed(e, 1, s, true)) return BGX_E_HIP;
            HIP_TRY(bgx_launch_mlp(&r, s));
            if (timed(e, 1, s, false)) return BGX_E_HIP;
            // reference-sampled mode (cfg.reply_sample > 0): keyed by the seed and the
            // lane block, salted per step by the engine's env-step counter
            const uint64_t skey = e->cfg.seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(e->cfg.lane_base + 1));
            if (e->cfg.k_top == 4) {
                HIP_TRY(bgx_launch_top5(e->reply_V, e->job_off, e->job_cnt, L * 4 * 21, nullptr, 0, L * 4 * 21,
                                        e->job_val, e->cfg.reply_sample, skey, e->stats, e->stats + 8, s));
            } else {
                HIP_TRY(bgx_launch_top5(e->reply_V, e->job_off, e->job_cnt, 0, e->ctr + C_FLAT, 21, e->jobs_cap,
                                        e->job_val, e->cfg.reply_sample, skey, e->stats, e->stats + 8, s));
            }
        }
        HIP_TRY(bgx_launch_select(&e->d, s));   // select + env step (one launch)
    }
    return BGX_OK;
}

// fused 1-ply: one persistent launch for all n_steps (bgx_fused.hip)
static int enqueue_fused(bgx_engine* e, int n_steps, hipStream_t s) {
    bgx::FusedArgs f{};
    f.e = e->d;
    f.cand = e->fcand;
    f.vbuf = e->fvbuf;
    f.t1cnt = e->ft1cnt;
    f.t1_ready = e->t1_ready ? 1 : 0;
    f.cap = e->fcap;
    f.n_steps = n_steps;
    f.wfrag = e->net->wfrag;
    f.rowc = e->net->rowc;
    f.b2 = e->net->b2;
    f.feat_scale = e->net->feat_scale;
    f.ws_global = e->ws;
    f.ws_blocks = e->ws_waves;
    f.ws_slots = e->ws_slots;
    f.ws_words_per_block = (size_t)5 * e->ws_slots;
    f.force_tier = e->force_tier;
    f.lanes_per_wg = e->fused_fl;
    if (e->cfg.balance) {   // n_steps x lanes lane-steps; a lane runs at most n + n/4 + 4 (ring headroom)
        f.budget = (long long)n_steps * (long long)e->cfg.lanes;
        const int headroom = e->cfg.ring - e->cfg.max_steps;
        const int cap = n_steps + n_steps / 4 + 4;
        f.n_cap = cap < headroom ? cap : headroom;
        f.budget_ctr = (unsigned long long*)(e->ctr + C_BUDGET);
    }
    {   // in-kernel harvest into the slot of the next ticket
        const int b = e->h_tickets % bgx_engine::NHB;
        f.hv_hdr = e->out_headers[b];
        f.hv_rec = e->out_records[b];
        f.hv_ep_cap = e->d.ep_cap;
        f.hv_rec_cap = (long long)e->cfg.lanes * e->cfg.ring;
        f.hv_ctr = e->fh_ctr + b;
        f.hv_next = e->fh_ctr + (b + 1) % bgx_engine::NHB;
        f.hv_flags = e->fh_ctr + bgx_engine::NHB + 1 + b;
        f.hv_next_flags = e->fh_ctr + bgx_engine::NHB + 1 + (b + 1) % bgx_engine::NHB;
        f.hv_commit = e->fh_ctr + 2 * bgx_engine::NHB + 1 + b;
        f.hv_next_commit = e->fh_ctr + 2 * bgx_engine::NHB + 1 + (b + 1) % bgx_engine::NHB;
        f.hv_info = e->d_info[b];
        f.hv_hinfo = e->h_info_dev + 4 * b;
        f.done_ctr = e->fh_ctr + bgx_engine::NHB;
    }
    if (e->prof_enabled) {
        if (!e->fprof) {
            if (dalloc(&e->fprof, (size_t)1024 * PROF_W)) return BGX_E_HIP;
            HIP_TRY(hipMemset(e->fprof, 0, (size_t)1024 * PROF_W * 8));
        }
        f.prof = e->fprof;
    }
    if (timed(e, 0, s, true)) return BGX_E_HIP;
    HIP_TRY(bgx_launch_fused(&f, s));
    e->t1_ready = true;   // the launch ends with every lane's next position expanded
    e->fh_launched = true;
    if (timed(e, 0, s, false)) return BGX_E_HIP;
    return BGX_OK;
}

int bgx_step(bgx_engine* e, int n_steps, void* stream) {
    return guarded("bgx_step", [&]() -> int {
        if (!e || n_steps < 0) return fail(BGX_E_ARG, "bgx_step: bad arguments");
        if (!e->net) return fail(BGX_E_STATE, "bgx_step: bgx_set_weights first");
        if (n_steps > e->cfg.ring - e->cfg.max_steps)
            return fail(BGX_E_ARG, "bgx_step: n_steps=%d > ring - max_steps = %d (harvest more often)", n_steps,
                        e->cfg.ring - e->cfg.max_steps);
        HIP_TRY(hipSetDevice(e->device));
        hipStream_t s = (hipStream_t)stream;
        // an enqueued harvest on another stream reads the rings and resets the
        // episode list: the step waits for it (an event, no host wait)
        if (e->h_tickets > 0 && e->hstream != s)
            HIP_TRY(hipStreamWaitEvent(s, e->hdone[(e->h_tickets - 1) % bgx_engine::NHB], 0));
        e->last = s;
        if (n_steps == 0) return BGX_OK;
        // timed runs launch directly (events between the kernels); otherwise the
        // n_steps sequence is one graph launch (kernel arguments are fixed for the
        // engine's lifetime; bgx_set_weights drops the graph: temperature is an argument)
        if (e->fused) return enqueue_fused(e, n_steps, s);
        if (e->timing || !e->use_graph) return enqueue_steps(e, n_steps, s);
        if (!e->gexec || e->g_steps != n_steps) {
            if (e->gexec) {
                HIP_TRY(hipGraphExecDestroy(e->gexec));
                e->gexec = nullptr;
            }
            if (!e->cap) HIP_TRY(hipStreamCreateWithFlags(&e->cap, hipStreamNonBlocking));
            HIP_TRY(hipStreamBeginCapture(e->cap, hipStreamCaptureModeRelaxed));
            const int rc = enqueue_steps(e, n_steps, e->cap);
            hipGraph_t g = nullptr;
            const hipError_t ec = hipStreamEndCapture(e->cap, &g);
            if (rc) {
                if (g) (void)hipGraphDestroy(g);
                return rc;
            }
            HIP_TRY(ec);
            const hipError_t ei = hipGraphInstantiate(&e->gexec, g, nullptr, nullptr, 0);
            (void)hipGraphDestroy(g);
            HIP_TRY(ei);
            e->g_steps = n_steps;
        }
        HIP_TRY(hipGraphLaunch(e->gexec, s));
        return BGX_OK;
    });
}

int bgx_sync(bgx_engine* e) {
    return guarded("bgx_sync", [&]() -> int {
        if (!e) return fail(BGX_E_ARG, "bgx_sync: null engine");
        HIP_TRY(hipSetDevice(e->device));
        HIP_TRY(hipStreamSynchronize(e->last));
        return check_flags(e);
    });
}

int bgx_harvest_enqueue(bgx_engine* e, int* ticket, void* stream) {
    return guarded("bgx_harvest_enqueue", [&]() -> int {
        if (!e || !ticket) return fail(BGX_E_ARG, "bgx_harvest_enqueue: null pointer");
        HIP_TRY(hipSetDevice(e->device));
        hipStream_t s = (hipStream_t)stream;
        // order after the engine's last step (another stream): an event, no host wait
        if (e->last != s) {
            if (!e->hev) HIP_TRY(hipEventCreateWithFlags(&e->hev, hipEventDisableTiming));
            HIP_TRY(hipEventRecord(e->hev, e->last));
            HIP_TRY(hipStreamWaitEvent(s, e->hev, 0));
        }
        const int t = e->h_tickets, b = t % bgx_engine::NHB;
        // offsets and totals on the device (harvest_scan_kernel, which also writes
        // {episodes, records, error flags} into host-mapped memory), then the copy
        // of the finished episodes' headers and records (a persistent grid that
        // reads the episode count on the device: no host round trip in between)
        if (e->fused) {
            // the fused launches since the last ticket harvested into slot b and
            // published its totals; with none, publish the (empty) slot here
            if (!e->fh_launched)
                HIP_TRY(bgx_launch_harvest_close(e->fh_ctr + 2 * bgx_engine::NHB + 1 + b,
                                                 e->fh_ctr + (b + 1) % bgx_engine::NHB,
                                                 e->fh_ctr + 2 * bgx_engine::NHB + 1 + (b + 1) % bgx_engine::NHB,
                                                 e->fh_ctr + bgx_engine::NHB + 1 + b,
                                                 e->fh_ctr + bgx_engine::NHB + 1 + (b + 1) % bgx_engine::NHB,
                                                 e->ctr + C_ERR, e->d_info[b], e->h_info_dev + 4 * b, s));
            e->fh_launched = false;
        } else {
            HIP_TRY(bgx_launch_harvest_scan(&e->d, e->d_offs[b], e->d_info[b], e->h_info_dev + 4 * b, s));
            HIP_TRY(bgx_launch_harvest_gather(&e->d, e->d_offs[b], e->d_info[b], e->out_headers[b], e->out_records[b],
                                              s));
        }
        HIP_TRY(hipEventRecord(e->hdone[b], s));
        e->hstream = s;
        e->h_tickets = t + 1;
        *ticket = t;
        return BGX_OK;
    });
}

// Wait for a harvest event: poll it for up to 2 ms (a short launch's harvest
// lands within that; a blocking wait adds the runtime's wake-up after the
// kernel ends), then block. BGX_SPIN_WAIT=0: block at once (A/B).
static hipError_t wait_event(hipEvent_t ev) {
    static const int spin = [] {
        const char* v = getenv("BGX_SPIN_WAIT");
        return v ? atoi(v) : 1;
    }();
    if (spin) {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            const hipError_t q = hipEventQuery(ev);
            if (q != hipErrorNotReady) return q;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(2000)) break;
        }
    }
    return hipEventSynchronize(ev);
}

int bgx_harvest_fetch(bgx_engine* e, int ticket, bgx_harvest_info* out) {
    return guarded("bgx_harvest_fetch", [&]() -> int {
        if (!e || !out) return fail(BGX_E_ARG, "bgx_harvest_fetch: null pointer");
        if (ticket < 0 || ticket >= e->h_tickets || ticket < e->h_tickets - 2)
            return fail(BGX_E_ARG, "bgx_harvest_fetch: ticket %d is not one of the last two harvests (%d enqueued)",
                        ticket, e->h_tickets);
        HIP_TRY(hipSetDevice(e->device));
        const int b = ticket % bgx_engine::NHB;
        HIP_TRY(wait_event(e->hdone[b]));
        // the ticket's own flags: its harvest (or the last launch before it)
        // moved them out of the engine word on the device, in stream order
        const uint32_t* info = e->h_info + 4 * b;
        const uint32_t flags = info[2];
        if (flags) return flag_error(flags);
        out->n_episodes = (int)info[0];
        out->n_records = (int)info[1];
        out->d_headers = e->out_headers[b];
        out->d_records = e->out_records[b];
        return BGX_OK;
    });
}

int bgx_harvest(bgx_engine* e, bgx_harvest_info* out, void* stream) {
    return guarded("bgx_harvest", [&]() -> int {
        int t = 0;
        if (int rc = bgx_harvest_enqueue(e, &t, stream)) return rc;
        return bgx_harvest_fetch(e, t, out);
    });
}

int bgx_get_stats(bgx_engine* e, bgx_stats* out) {
    return guarded("bgx_get_stats", [&]() -> int {
        if (!e || !out) return fail(BGX_E_ARG, "bgx_get_stats: null pointer");
        HIP_TRY(hipSetDevice(e->device));
        if (e->last) HIP_TRY(hipStreamSynchronize(e->last));
        std::vector<unsigned long long> st(kStatWords);
        HIP_TRY(hipMemcpy(st.data(), e->stats, kStatWords * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        for (int i = 8; i < kStatWords; ++i) st[7] += st[i];   // the top-5 launch's per-wave record counts
        // decisions = records written, episodes = games finished: the lanes' own counters
        const int L = e->cfg.lanes;
        std::vector<uint32_t> rec(L), epi(L);
        HIP_TRY(hipMemcpy(rec.data(), e->d.rec_count, (size_t)L * 4, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(epi.data(), e->d.epi, (size_t)L * 4, hipMemcpyDeviceToHost));
        unsigned long long dec = 0, eps = 0;
        for (int i = 0; i < L; ++i) {
            dec += rec[i];
            eps += epi[i];
        }
        out->env_steps = st[0];
        out->decisions = dec;
        out->episodes = eps;
        out->value_rows = st[3];
        out->movegen_jobs = st[4];
        out->fallback_jobs = st[5];
        // 2-ply reply rows reserved minus the records written into them; a step
        // stopped between the top-5 launch (st[7]) and the step kernel (st[6])
        // would make the difference negative, so clamp at zero
        out->gap_rows = st[6] > st[7] ? st[6] - st[7] : 0;
        return BGX_OK;
    });
}

int bgx_engine_peek(bgx_engine* e, int buf, void* h_out, uint64_t bytes, uint64_t* needed) {
    return guarded("bgx_engine_peek", [&]() -> int {
        if (!e) return fail(BGX_E_ARG, "bgx_engine_peek: null engine");
        const size_t L = (size_t)e->cfg.lanes;
        const void* src = nullptr;
        size_t n = 0;
        switch (buf) {
        case BGX_PEEK_LANE_ROWS: src = e->rows; n = L * 8 * 4; break;
        case BGX_PEEK_PLAYER: src = e->d.player; n = L; break;
        case BGX_PEEK_DICE: src = e->d.dice; n = 2 * L; break;
        case BGX_PEEK_CAND_OFF: src = e->cand_off; n = L * 4; break;
        case BGX_PEEK_CAND_CNT: src = e->cand_cnt; n = L * 4; break;
        case BGX_PEEK_CAND_ROWS: src = e->rows + L * 8; n = (size_t)e->cand_cap * 8 * 4; break;
        case BGX_PEEK_VALUES: src = e->V; n = (L + (size_t)e->cand_cap) * 4; break;
        case BGX_PEEK_SEL: src = e->sel; n = e->sel ? 4 * L * 4 : 0; break;
        case BGX_PEEK_JOB_VAL: src = e->job_val; n = e->job_val ? (size_t)e->jobs_cap * 4 : 0; break;
        default: return fail(BGX_E_ARG, "bgx_engine_peek: unknown buffer %d", buf);
        }
        if (e->fused && buf != BGX_PEEK_PLAYER && buf != BGX_PEEK_DICE)
            return fail(BGX_E_STATE, "bgx_engine_peek: buffer %d is not kept by the fused engine", buf);
        if (!src || n == 0) return fail(BGX_E_STATE, "bgx_engine_peek: buffer %d not allocated (ply %d)", buf, e->cfg.ply);
        if (needed) *needed = n;
        if (!h_out) return BGX_OK;
        if (bytes < n) return fail(BGX_E_ARG, "bgx_engine_peek: %llu bytes < %zu", (unsigned long long)bytes, n);
        HIP_TRY(hipSetDevice(e->device));
        if (e->last) HIP_TRY(hipStreamSynchronize(e->last));
        HIP_TRY(hipMemcpy(h_out, src, n, hipMemcpyDeviceToHost));
        return BGX_OK;
    });
}

int bgx_set_timing(bgx_engine* e, int enabled) {
    return guarded("bgx_set_timing", [&]() -> int {
        if (!e) return fail(BGX_E_ARG, "bgx_set_timing: null engine");
        HIP_TRY(hipSetDevice(e->device));
        if (e->last) HIP_TRY(hipStreamSynchronize(e->last));
        for (hipEvent_t ev : e->ev) hipEventDestroy(ev);
        e->ev.clear();
        e->ev_kind.clear();
        e->ms_mg = e->ms_mlp = 0;
        e->n_mg = e->n_mlp = 0;
        e->timing = enabled != 0;
        return BGX_OK;
    });
}

int bgx_get_timing(bgx_engine* e, double* ms_movegen, int* n_movegen, double* ms_mlp, int* n_mlp) {
    return guarded("bgx_get_timing", [&]() -> int {
        if (!e) return fail(BGX_E_ARG, "bgx_get_timing: null engine");
        HIP_TRY(hipSetDevice(e->device));
        if (e->last) HIP_TRY(hipStreamSynchronize(e->last));
        for (size_t i = 0; i + 1 < e->ev.size(); i += 2) {
            float ms = 0;
            HIP_TRY(hipEventElapsedTime(&ms, e->ev[i], e->ev[i + 1]));
            if (e->ev_kind[i] == 0) { e->ms_mg += ms; e->n_mg++; }
            else { e->ms_mlp += ms; e->n_mlp++; }
        }
        for (hipEvent_t ev : e->ev) hipEventDestroy(ev);
        e->ev.clear();
        e->ev_kind.clear();
        if (ms_movegen) *ms_movegen = e->ms_mg;
        if (n_movegen) *n_movegen = e->n_mg;
        if (ms_mlp) *ms_mlp = e->ms_mlp;
        if (n_mlp) *n_mlp = e->n_mlp;
        return BGX_OK;
    });
}

}  // extern "C"
