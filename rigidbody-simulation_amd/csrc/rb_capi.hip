// rb_capi.hip — implementation of include/rbhip.h.
//
// A world owns its device buffers — struct-of-arrays state, replicated
// constants, two ping-pong position snapshots (which double as the
// replicated exchange buffer of sharded worlds) and two alternating
// broadphase tables (generation-tagged bucket lines, never cleared) — and
// enqueues all work on one HIP stream.  A step's buffers are fixed by the
// step counter's parity (and table generations live on the device), so
// multi-step calls are captured once per parity into a hipGraph (one kernel
// node per step) and replayed.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>   // types only: RCCL is dlopen'ed by the sharded path

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/rbhip.h"
#include "rb_internal.hpp"

// Threads.  A graph capture on one thread's stream is invalidated by a
// null-stream or device-wide call (hipMalloc, hipMemset, hipMemcpy, hipFree,
// ...) that another thread makes on the same device meanwhile, and that call
// fails too (seen with two threads creating, stepping and destroying their
// own worlds).  So every entry point runs inside an ApiScope of its world's
// device, and a capture (graph_replay) inside a CaptureScope: a capture on
// device d starts once no other thread is inside an entry point on d (other
// than capturing too), and no entry point on d starts while a capture on d
// runs.  Captures of several threads may overlap; a thread working on one
// device never waits for a capture on another.  Entry points with no device
// (rb_comm_unique_id) or no valid world gate every device.
namespace {
constexpr int GATE_DEVICES = 64;
struct Gate {
    std::mutex m;
    std::condition_variable cv;
    int active[GATE_DEVICES] = {};      // threads inside an entry point on device d, not capturing
    int capturing[GATE_DEVICES] = {};   // threads inside a capture on device d
    int active_all = 0;                 // threads inside a device-less entry point
    int capturing_any = 0;
};
Gate &gate() {
    static Gate g;
    return g;
}
int gate_dev(int d) { return d >= 0 && d < GATE_DEVICES ? d : -1; }
thread_local int t_api_depth = 0;
thread_local int t_api_dev = -1;
struct ApiScope {
    explicit ApiScope(int device) {
        if (t_api_depth++ == 0) {
            const int d = gate_dev(device);
            t_api_dev = d;
            Gate &g = gate();
            std::unique_lock<std::mutex> l(g.m);
            g.cv.wait(l, [&] { return d < 0 ? g.capturing_any == 0 : g.capturing[d] == 0; });
            if (d < 0) ++g.active_all; else ++g.active[d];
        }
    }
    ~ApiScope() {
        if (--t_api_depth == 0) {
            Gate &g = gate();
            std::lock_guard<std::mutex> l(g.m);
            if (t_api_dev < 0) --g.active_all; else --g.active[t_api_dev];
            g.cv.notify_all();
        }
    }
    ApiScope(const ApiScope &) = delete;
    ApiScope &operator=(const ApiScope &) = delete;
};
struct CaptureScope {   // (inside an ApiScope of a device: the capture's)
    int d;
    CaptureScope() : d(t_api_dev < 0 ? 0 : t_api_dev) {
        Gate &g = gate();
        std::unique_lock<std::mutex> l(g.m);
        if (t_api_dev < 0) --g.active_all; else --g.active[d];
        ++g.capturing[d];
        ++g.capturing_any;
        g.cv.wait(l, [&] { return g.active[d] == 0 && g.active_all == 0; });
    }
    ~CaptureScope() {
        Gate &g = gate();
        std::unique_lock<std::mutex> l(g.m);
        --g.capturing[d];
        --g.capturing_any;
        g.cv.notify_all();
        g.cv.wait(l, [&] { return g.capturing[d] == 0; });
        if (t_api_dev < 0) ++g.active_all; else ++g.active[d];
    }
    CaptureScope(const CaptureScope &) = delete;
    CaptureScope &operator=(const CaptureScope &) = delete;
};
}  // namespace

using namespace rb;

static_assert(CK_SPHERE_BOX == RB_CK_SPHERE_BOX && CK_BOX_BOX0 == RB_CK_BOX_BOX0 && CK_BOX_EDGE == RB_CK_BOX_EDGE,
              "contact kinds");

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(e_ == hipErrorOutOfMemory ? RB_ENOMEM : RB_ENODEV, "%s: %s (%s:%d)", #expr, \
                        hipGetErrorString(e_), __FILE__, __LINE__);                           \
    } while (0)

// Every fill and copy of a world's buffers is enqueued on the world's own
// stream (w->stream), so it is ordered with the world's kernels by
// construction: a null-stream hipMemset / hipMemcpy is not ordered with a
// non-blocking stream (one once zeroed contact counts a step had just
// recorded), and a null-stream call also invalidates another thread's
// graph capture on the device.  Copies from or into host memory the caller
// frees on return end with a sync of that stream.
#define WCHK(expr)                                                                            \
    do {                                                                                      \
        if (int rc_ = (expr)) return rc_;                                                     \
    } while (0)

int64_t next_pow2(int64_t v) {
    int64_t p = 1;
    while (p < v) p <<= 1;
    return p;
}

int err_to_code(int32_t bits) {
    if (bits & ERR_EXCHANGE) return fail(RB_ENODEV, "device: peer-to-peer exchange timed out (a peer rank did not reach the step)");
    if (bits & ERR_HALO_MOVE)
        return fail(RB_EDOM, "device: a body moved more than one broadphase cell in one step (the halo exchange "
                             "cannot guarantee its partners; use full peer reads: rb_p2p_halo(w, 0))");
    if (bits & ERR_DOMAIN) return fail(RB_EDOM, "device: non-finite or out-of-range body position");
    if (bits & ERR_UNSUPPORTED)
        return fail(RB_EUNSUPPORTED, "device: box-involved pair within contact range with no box kernel to take it");
    if (bits & ERR_PARTNER_OVERFLOW) return fail(RB_EOVERFLOW, "device: a body has more sphere partners than max_partners");
    if (bits & ERR_BUCKET_OVERFLOW) return fail(RB_EOVERFLOW, "device: more than 30 bodies hashed to one broadphase bucket");
    return RB_OK;
}

}  // namespace

struct rb_world {
    int dtype = RB_F64, esz = 8, device = 0;
    hipStream_t stream = nullptr, own_stream = nullptr, cap_stream = nullptr;
    int64_t N = 0, S = 0, Npad = 0, lo = 0;
    int32_t n_local = 0, P = 1, rank = 0;
    int32_t n_planes = 0, oriented = 1, maxp = 16, maxrec = 0;
    // owned bodies up to which the cooperative search is used: above it
    // the wide form (with its helper wave) is faster (19,600: 14.4 vs 12.1
    // us; 16,384: 11.1 vs 11.3, 12,100: 10.4 vs 11.5 the other way;
    // profiles/r03/wide_help/ab_thresh_flat.txt)
    int64_t coop_max = 16384;
    // above coop_max, up to which the wide one-lane form is used; with its
    // helper wave it is at least as fast as the one-lane form at every size
    // measured (131k / 262k equal, 524k 0.116 -> 0.102 ms, 1M 0.236 ->
    // 0.216, 4M 0.876 -> 0.841; profiles/r03/wide_help/ab_large2.txt), so
    // the one-lane form only runs on request (RBHIP_WIDE_MAX_BODIES)
    int64_t wide_max = INT64_MAX;
    // owned bodies up to which the cooperative form runs with a helper wave
    // per workgroup (inv(I_w), gravity and plane contacts off the body
    // lanes' chain): 4k 8.1 -> 7.4 us, 8k 9.6 -> 8.6; 16k 11.0 -> 11.9 the
    // other way (its waves then share SIMDs)
    int64_t help_max = 12288;
    // the wide form with a helper wave per workgroup (inv(I_w), gravity,
    // plane contacts and the state / constant loads off the body wave;
    // A/B steps 261-460, profiles/r03/wide_help_ab.txt): 32k 13.6 -> 12.9
    // us, C3 16.8 -> 16.1, C4 15.4 -> 14.9, C5 (16,384 cubes) 12.1 -> 9.6
    bool wide_help = true;
    double planes[RB_MAX_PLANES][6] = {};
    double g[3] = {};
    double inv_cs = 1.0;
    double rmax = 0.0;             // largest bounding radius
    bool all_spheres = true;
    bool boxes = false;            // box-capable step kernels (any box body; sharded worlds exchange orientations)
    // contact law (rb_set_contact_law)
    int32_t law = RB_LAW_MUJOCO;
    double tol = 0.01;
    double prm_dt = 0, prm_e = 0, prm_mu = 0;   // the ground phase held in the snapshots (two-ball law)
    int64_t H = 4096;
    int64_t hmax = 4096;           // the table's growth limit (RBHIP_HASH_MAX_BYTES)
    int32_t group = 0;             // Grid::super: bucket grouping shape (x | y << 4 | z << 8 bits)
    bool fit_valid = false;        // fit_period: the group box (and layout) the last fit was made for
    int64_t fit_key[7] = {};
    int64_t bytes_per_body_step = 0;
    std::vector<double> bound;     // host copy of every body's bounding radius (rb_set_state's snapshot rows)
    // device memory
    void *snap[2] = {};        // [Npad] Snap<T>: (x, y, z, bound radius), ping-pong
    void *qsnap[2] = {};       // boxes: [Npad][4] step-start orientations, ping-pong with snap
    int32_t *defer_q = nullptr;    // boxes: [S] bodies the step kernel defers to the box kernel
    int32_t *defer_cnt = nullptr;  // boxes: [2] queue lengths by step parity
    // box worlds, one rank: chunks of steps replay optimistically WITHOUT the
    // box kernel (an idle one still costs a kernel boundary per step); the
    // step kernels then only count deferrals, and a chunk that deferred any
    // body is rolled back to its start and replayed with the box kernel
    bool box_opt = true;           // RBHIP_BOX_OPTIMISTIC=0: always launch the box kernel
    bool box_kernel_on = true;     // launch_one: the box kernel follows the step kernel
    int32_t box_backoff = 0;       // chunks to run with the box kernel after a rollback (doubles)
    int32_t box_skip = 0;          // of which left
    void *opt_save = nullptr;      // chunk-start copy: state rows, snapshot, orientations, error word
    int32_t *defer_host = nullptr; // pinned [2]
    int64_t box_stats[2] = {};     // optimistic chunks, rollbacks
    bool sync_call = false;        // inside rb_step (synchronous): long chunks are guarded
    int64_t refits = 0;            // layout refits after a bucket overflow (rolled back, replayed)
    int64_t table_grows = 0;       // of which with the table doubled
    int64_t partner_grows = 0;     // max_partners raised 16 -> 32 after a partner overflow
    int32_t diag_overflow = 0;     // RBHIP_DIAG_OVERFLOW=n (tests): the next n guarded chunk checks
                                   // report a bucket overflow (the roll-back / refit / growth path)
    void *state = nullptr;     // 13 x S  (qw qx qy qz vx vy vz wx wy wz px py pz)
    void *vel[2] = {};         // two-ball law: [Npad] Vel<T>, ping-pong with the snapshots
    void *consts = nullptr;    // 8 x Npad (mass ix iy iz sx sy sz bound)
    int32_t *kind = nullptr;   // Npad
    void *xfrc = nullptr;      // 6 x S or null
    uint32_t *ids[2] = {};     // [H][LINE_WORDS] bucket blocks (rb_internal.hpp Table; alternate with the snapshots)
    uint32_t *spill[2] = {};   // [SPILL_LINES x SPILL_LINE_WORDS] ids past full buckets, per table
    void *pos[2] = {};         // [H][LINE_WORDS] Snap<T> bucket slot snapshots
    uint32_t *gen = nullptr;   // [2] generation of the table of each step parity (rb_internal.hpp Table)
    uint32_t gen_off = 1;      // generation of step c's table = gen_off + c (host bookkeeping; only grows)
    int32_t *plist = nullptr;      // split form: [MAXP][S] sorted partner ids
    int32_t *plist_cnt = nullptr;  // split form: [S] partner counts
    int32_t *err = nullptr;
    int32_t *err_host = nullptr;   // pinned, device-mapped (publish_err_kernel writes it)
    int32_t *err_host_d = nullptr;
    // err_host holds the error word as of all error-writing work enqueued so
    // far: set by a graph launch (every captured graph ends in
    // publish_err_kernel), cleared by every builder of kernel parameters that
    // carry the error word and by every write to it.  rb_sync / rb_step then
    // only synchronise the stream.
    bool err_pub = false;
    ncclComm_t comm = nullptr;     // rb_shard_comm_init: the in-library exchange
    // peer-to-peer exchange (rb_p2p_connect)
    bool p2p = false;
    int64_t *flags = nullptr;      // the mailbox (MailLayout, uncached); starts with flags[P]: peer q
                                   // writes slot q when its step is done
    bool halo = false;             // rb_p2p_halo: push only the bodies a peer can reach
    int32_t *bounds = nullptr;     // peer-to-peer: [2][BOUND_COPIES][BOUND_STRIDE] own cell bounds (step parity)
    int32_t *push_cnt = nullptr;   // halo: [P] bodies pushed to each peer this step
    int64_t *halo_e = nullptr;     // halo: the epoch the next step kernel's pushes test against
    int64_t *epoch = nullptr;      // steps taken since connect (advanced by the step kernel)
    void **peer_snap_dev = nullptr;       // [2][P] device array: each rank's snapshot buffers
    void **peer_quat_dev = nullptr;       // box worlds: [2][P] each rank's orientation snapshots
    int64_t **peer_flags_dev = nullptr;   // [P] device array: each rank's flag array
    std::vector<void *> ipc_opened;       // peer mappings to close
    // recording
    bool record = false;
    int32_t *rec_count = nullptr, *rec_partner = nullptr, *rec_kind = nullptr;
    void *rec_dist = nullptr;
    // stepping state: step counter c; bucket counts rotate mod 3, snapshots
    // and bucket slots mod 2
    int64_t c = 0;
    bool primed = false;
    // captured K-step graphs, least recently used evicted past GRAPH_CACHE_MAX
    // entries (a caller stepping varying chunk lengths would otherwise keep
    // accumulating executables)
    struct GraphEntry { hipGraphExec_t ex; uint64_t used; };
    std::map<std::tuple<int64_t, int, double, double, double, double, int>, GraphEntry> graphs;
    uint64_t graph_tick = 0;
    // the boundary's staging (rb_set_state / rb_get_state): pinned host rows
    // in the caller's layout and their device twins, moved with one DMA each
    // way and transposed by a kernel.  The staging mirrors the device state
    // while mirror_version == state_version (every change of the state bumps
    // it): an rb_set_state with exactly those bytes is then a no-op
    double *io_q_h = nullptr, *io_v_h = nullptr;   // pinned [N][7], [N][6]
    double *io_q_hd = nullptr, *io_v_hd = nullptr; // the same pinned rows, device-mapped (rb_get_state's kernel writes them)
    hipEvent_t io_ev[4] = {};      // rb_get_state (RBHIP_IO_OUT=1): the download in chunks, each copied out as it lands
    double *io_q_d = nullptr, *io_v_d = nullptr;   // device
    int64_t state_version = 0, mirror_version = -1;
    int64_t io_stats[2] = {};      // rb_set_state calls skipped (unchanged), uploads
    // kernel timing
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> tev;
    double t_sum_ms = 0;
    int64_t t_n = 0;

    // cell-ordered tile form (rb_tiles.hip): sphere worlds on
    // one rank step in tile slots when eligible (tile_eligible).  The bins
    // (the state sorted by column, per step parity) are a cache of the
    // id-ordered state rows and snapshot: built from them at the first tile
    // run, carried from run to run, written back at the end of each run by
    // the unbin kernel — only if no step of it raised ERR_TILE, so that a
    // failed run leaves the id-ordered state at the start of the first
    // failed run, which the host replays with the hashed-cell forms
    // (tile_finish) at the next sync point.
    int tile_mode = -1;            // RBHIP_TILE: 0 off, 1 every eligible world, -1 auto (default: >= tile_min_bodies, off after a roll-back)
    int tile_mode_init = -1;       // the mode at creation (auto: re-armed by an rb_set_state that uploads)
    int32_t tile_ntypes = 0;       // distinct (m, I) of the bodies when <= TILE_TYPES (else 0: no tile form)
    double tile_type_val[TILE_TYPES][4] = {};   // m ix iy iz of each type
    uint8_t *tile_type_of = nullptr;   // [N]
    int64_t tile_min_bodies = 65537;    // (the hashed forms win up to C3's 65,536 bodies, the tile form above: DESIGN §4.1)
    int32_t tile_tc = 0, tile_ntx = 0, tile_nty = 0, tile_cap = TILE_THREADS;
    bool tile_fit_valid = false;
    int tile_valid_sp = -1;        // the bins of this parity hold the state at step c (-1: no bins)
    void *tile_mem = nullptr;      // bins x 2 (column tables, positions, ids, state), far lists x 2
    size_t tile_mem_bytes = 0;
    int32_t *tile_fill = nullptr;  // build scratch [slots][TILE_OFFW]
    uint32_t *tile_gen = nullptr;  // [2] generation of each parity's bins (far-list tags)
    int32_t *tile_why = nullptr;   // TILE_WHY_* bits raised (device)
    unsigned long long *tile_commits = nullptr;   // runs committed by the unbin kernel (device)
    int64_t *tile_host = nullptr;  // pinned: err, why, commits
    int64_t *tile_pub_host = nullptr, *tile_pub_host_d = nullptr;   // pinned, mapped: why, commits (tile graphs' publish)
    bool tile_pub = false;         // err_pub, and the last graph was a tile run's (tile_pub_host is current)
    unsigned long long tile_commits_seen = 0;
    // a tile run whose check waits for the next sync point
    struct TileRun { int64_t c0, n; double dt, e, mu, thr; };
    std::vector<TileRun> tile_pending;    // runs enqueued since the last check
    int64_t tile_stats[4] = {};    // runs, steps committed, runs rolled back, bin builds
    int32_t tile_why_seen = 0;     // why bits of the runs rolled back (OR)
    int32_t tile_backoff = 0, tile_skip = 0;   // eligible runs to step hashed after a roll-back (doubling)
    bool tile_replaying = false;   // tile_finish's replay steps hashed


    int sp() const { return (int)(c % 2); }
};

extern "C" {
static void fit_period(rb_world *w, const double *qpos, bool force = false);   // (below)
}

namespace {
// stream-ordered fills and copies of world buffers (WCHK above)
int wfill(rb_world *w, void *dst, int value, size_t bytes) {
    HIPCHK(hipMemsetAsync(dst, value, bytes, w->stream));
    return RB_OK;
}
// from host memory the caller may free on return: waits for the copy
int wput(rb_world *w, void *dst, const void *src, size_t bytes) {
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, w->stream));
    HIPCHK(hipStreamSynchronize(w->stream));
    return RB_OK;
}
// into host memory: ordered after the world's work so far, waited for
int wget(rb_world *w, void *dst, const void *src, size_t bytes) {
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, w->stream));
    HIPCHK(hipStreamSynchronize(w->stream));
    return RB_OK;
}
}  // namespace

namespace {

template <typename T> T *dp(void *p, int64_t off) { return reinterpret_cast<T *>(p) + off; }

template <typename T> Grid<T> make_grid(const rb_world *w) {
    Grid<T> g;
    g.inv_cs = (T)w->inv_cs;
    g.hmask = (uint32_t)(w->H - 1);
    g.H = (int32_t)w->H;
    g.super = w->group;
    return g;
}

// the broadphase of the steps of parity sp
template <typename T> Table<T> table(const rb_world *w, int sp) {
    return Table<T>{w->ids[sp], w->pos[sp] ? dp<Snap<T>>(w->pos[sp], 0) : nullptr, w->gen + sp, w->spill[sp]};
}

// parameters of the step with counter value c
template <typename T> StepParams<T> make_step(rb_world *w, int64_t c, double dt, double e, double mu, double thr,
                                              bool insert_next) {
    w->err_pub = false;
    StepParams<T> p{};
    p.n_global = w->N;
    p.n_local = w->n_local;
    p.lo = (int32_t)w->lo;
    p.S = (int32_t)w->S;
    p.st.base = dp<T>(w->state, 0);
    p.st.S = w->S;
    p.cs.base = dp<T>(w->consts, 0);
    p.cs.Npad = w->Npad;
    p.cs.kind = w->kind;
    p.xfrc = w->xfrc ? dp<T>(w->xfrc, 0) : nullptr;
    p.n_planes = w->n_planes;
    for (int k = 0; k < w->n_planes; ++k)
        for (int d = 0; d < 3; ++d) { p.pn[k][d] = (T)w->planes[k][d]; p.pp[k][d] = (T)w->planes[k][3 + d]; }
    for (int d = 0; d < 3; ++d) p.g[d] = (T)w->g[d];
    p.dt = (T)dt; p.e = (T)e; p.mu = (T)mu; p.thr = (T)thr;
    p.oriented = w->oriented;
    p.grid = make_grid<T>(w);
    const int sp = (int)(c % 2);
    p.snap_cur = dp<Snap<T>>(w->snap[sp], 0);
    p.snap_next = dp<Snap<T>>(w->snap[1 - sp], 0);
    p.cur = table<T>(w, sp);
    p.next = insert_next ? table<T>(w, 1 - sp) : Table<T>{nullptr, nullptr, nullptr, nullptr};
    p.err = w->err;
    p.epoch = w->p2p ? w->epoch : nullptr;
    p.bounds = w->p2p ? w->bounds + (c % 2) * BOUND_COPIES * BOUND_STRIDE : nullptr;   // (peer-to-peer: both modes filter by them)
    if (w->p2p && w->halo) {                     // the step kernels push to the peers (rb_halo.hpp)
        p.halo.peer_mail = reinterpret_cast<char *const *>(w->peer_flags_dev);
        p.halo.mail = reinterpret_cast<const char *>(w->flags);
        p.halo.push_cnt = w->push_cnt;
        p.halo.halo_e = w->halo_e;
        p.halo.lay = MailLayout::make(w->P, w->S, w->esz, w->boxes);
        p.halo.S = w->S;
        p.halo.timeout_ticks = 500000000;        // 5 s at 100 MHz
        p.halo.rank = (int32_t)w->rank;
        p.halo.P = (int32_t)w->P;
    }
    p.plist = w->plist;
    p.plist_cnt = w->plist_cnt;
    if (w->vel[0]) {
        p.vel_cur = dp<Vel<T>>(w->vel[sp], 0);
        p.vel_next = dp<Vel<T>>(w->vel[1 - sp], 0);
    }
    p.tol = (T)w->tol;
    p.ground = w->n_planes > 0;
    if (w->boxes) {
        p.quat_cur = dp<T>(w->qsnap[sp], 0);
        p.quat_next = dp<T>(w->qsnap[1 - sp], 0);
        p.defer_q = w->defer_q;
        p.defer_cnt = w->defer_cnt + sp;
        p.defer_reset = w->defer_cnt + (1 - sp);
    }
    if (w->record) {
        p.rec_count = w->rec_count; p.rec_partner = w->rec_partner; p.rec_kind = w->rec_kind;
        p.rec_dist = dp<T>(w->rec_dist, 0);
        p.maxrec = w->maxrec;
    }
    return p;
}

template <typename T> InsertParams<T> make_insert(rb_world *w, int sp, int64_t first, int64_t count,
                                                  int64_t skip_lo, int64_t skip_hi) {
    w->err_pub = false;
    InsertParams<T> ip{};
    ip.snap = dp<Snap<T>>(w->snap[sp], 0);
    ip.kind = w->kind;
    ip.first = first; ip.count = count; ip.skip_lo = skip_lo; ip.skip_hi = skip_hi;
    ip.grid = make_grid<T>(w);
    ip.tab = table<T>(w, sp);
    ip.err = w->err;
    return ip;
}

// (re)build the current table from every body's snapshot; under the
// two-ball law first run the coming step's ground phase from the true state
// (it depends on dt, e, mu: remembered, and re-primed when they change)
int prime(rb_world *w, double dt = 0, double e = 0, double mu = 0) {
    if (w->law == RB_LAW_BALLS) {
        hipError_t r;
        if (w->dtype == RB_F64) {
            StepParams<double> p = make_step<double>(w, w->c, dt, e, mu, 0.0, false);
            p.snap_next = dp<Snap<double>>(w->snap[w->sp()], 0);
            p.vel_next = dp<Vel<double>>(w->vel[w->sp()], 0);
            r = launch_ball_prime<double>(p, w->stream);
        } else {
            StepParams<float> p = make_step<float>(w, w->c, dt, e, mu, 0.0, false);
            p.snap_next = dp<Snap<float>>(w->snap[w->sp()], 0);
            p.vel_next = dp<Vel<float>>(w->vel[w->sp()], 0);
            r = launch_ball_prime<float>(p, w->stream);
        }
        HIPCHK(r);
        w->prm_dt = dt; w->prm_e = e; w->prm_mu = mu;
    }
    // a fresh table: a generation above every one used so far
    w->gen_off += 1;
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)(w->gen + w->sp()), (int)(w->gen_off + (uint32_t)w->c), 1, w->stream));
    hipError_t ie = w->dtype == RB_F64
                        ? launch_insert<double>(make_insert<double>(w, w->sp(), 0, w->N, 0, 0), w->stream)
                        : launch_insert<float>(make_insert<float>(w, w->sp(), 0, w->N, 0, 0), w->stream);
    HIPCHK(ie);
    w->primed = true;
    return RB_OK;
}

// the per-step kernel form of this world
int step_form(const rb_world *w) {
    return w->n_local <= w->coop_max ? (w->n_local <= w->help_max ? FORM_COOP_HELP : FORM_COOP)
           : w->n_local <= w->wide_max ? (w->wide_help ? FORM_WIDE_HELP : FORM_WIDE) : FORM_ONE;
}

int launch_one(rb_world *w, hipStream_t s, int64_t c, double dt, double e, double mu, double thr) {
    hipError_t r;
    if (w->law == RB_LAW_BALLS) {
        if (w->dtype == RB_F64) r = launch_ball_step<double>(make_step<double>(w, c, dt, e, mu, thr, true), w->maxp, s);
        else r = launch_ball_step<float>(make_step<float>(w, c, dt, e, mu, thr, true), w->maxp, s);
        HIPCHK(r);
        return RB_OK;
    }
    const int form = step_form(w);
    const bool boxes = w->boxes && w->box_kernel_on;
    if (w->dtype == RB_F64) r = launch_step<double>(make_step<double>(w, c, dt, e, mu, thr, true), w->maxp, form, boxes, s);
    else r = launch_step<float>(make_step<float>(w, c, dt, e, mu, thr, true), w->maxp, form, boxes, s);
    HIPCHK(r);
    return RB_OK;
}

int read_err(rb_world *w) {
    // the word reaches pinned host memory through publish_err_kernel: at the
    // end of the last graph, or enqueued here when other error-writing work
    // followed it (a separate launch costs ~9 us at a sync)
    if (!w->err_pub) HIPCHK(launch_publish_err(w->err, w->err_host_d, w->stream));
    HIPCHK(hipStreamSynchronize(w->stream));
    const int32_t bits = __atomic_load_n(w->err_host, __ATOMIC_ACQUIRE);
    if (bits) {
        w->err_pub = false;
        HIPCHK(hipMemsetAsync(w->err, 0, sizeof(int32_t), w->stream));
        HIPCHK(hipStreamSynchronize(w->stream));
        return err_to_code(bits);
    }
    return RB_OK;
}

int collect_timing(rb_world *w) {
    if (w->tev.empty()) return RB_OK;
    HIPCHK(hipStreamSynchronize(w->stream));
    for (auto &pr : w->tev) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, pr.first, pr.second));
        w->t_sum_ms += ms;
        w->t_n += 1;
        (void)hipEventDestroy(pr.first);
        (void)hipEventDestroy(pr.second);
    }
    w->tev.clear();
    return RB_OK;
}

int timed_launch(rb_world *w, double dt, double e, double mu, double thr) {
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    HIPCHK(hipEventRecord(a, w->stream));
    int rc = launch_one(w, w->stream, w->c, dt, e, mu, thr);
    if (rc) return rc;
    HIPCHK(hipEventRecord(b, w->stream));
    w->tev.emplace_back(a, b);
    if (w->tev.size() >= 4096) return collect_timing(w);
    return RB_OK;
}

// RCCL, loaded at first use: only the in-library exchange of sharded worlds
// needs it (and in a torch process the already-loaded copy is reused)
struct Rccl {
    bool tried = false, ok = false;
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
};
Rccl &rccl() {
    static Rccl r;
    if (r.tried) return r;
    r.tried = true;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return r;
    r.GetUniqueId = (decltype(r.GetUniqueId))dlsym(h, "ncclGetUniqueId");
    r.CommInitRank = (decltype(r.CommInitRank))dlsym(h, "ncclCommInitRank");
    r.AllGather = (decltype(r.AllGather))dlsym(h, "ncclAllGather");
    r.CommDestroy = (decltype(r.CommDestroy))dlsym(h, "ncclCommDestroy");
    r.GetErrorString = (decltype(r.GetErrorString))dlsym(h, "ncclGetErrorString");
    r.ok = r.GetUniqueId && r.CommInitRank && r.AllGather && r.CommDestroy && r.GetErrorString;
    return r;
}

// the peer-to-peer exchange of the next snapshot and table (parity nsp)
template <typename T> P2PParams<T> make_p2p(rb_world *w, int64_t c, int nsp) {
    w->err_pub = false;
    P2PParams<T> pp{};
    pp.ins = make_insert<T>(w, nsp, 0, w->N, w->lo, w->lo + w->n_local);
    pp.dst = dp<Snap<T>>(w->snap[nsp], 0);
    pp.peer_snap = reinterpret_cast<const Snap<T> *const *>(w->peer_snap_dev + (size_t)nsp * w->P);
    pp.peer_flags = w->peer_flags_dev;
    pp.flags = w->flags;
    pp.epoch = w->epoch;
    pp.rank = (int32_t)w->rank;
    pp.P = (int32_t)w->P;
    pp.S = w->S;
    pp.timeout_ticks = 500000000;      // 5 s at 100 MHz
    pp.bounds = w->bounds + (c % 2) * BOUND_COPIES * BOUND_STRIDE;
    pp.bounds_reset = w->bounds + ((c + 1) % 2) * BOUND_COPIES * BOUND_STRIDE;
    if (w->boxes) {
        pp.peer_quat = reinterpret_cast<const T *const *>(w->peer_quat_dev + (size_t)nsp * w->P);
        pp.qdst = dp<T>(w->qsnap[nsp], 0);
    }
    return pp;
}

// the halo exchange after the step kernel of step c (next snapshot and table nsp)
template <typename T> HaloParams<T> make_halo(rb_world *w, int64_t c, int nsp) {
    w->err_pub = false;
    HaloParams<T> hp{};
    hp.ins = make_insert<T>(w, nsp, 0, 0, 0, 0);
    hp.dst = dp<Snap<T>>(w->snap[nsp], 0);
    hp.bounds = w->bounds + (c % 2) * BOUND_COPIES * BOUND_STRIDE;
    hp.bounds_reset = w->bounds + ((c + 1) % 2) * BOUND_COPIES * BOUND_STRIDE;
    hp.push_cnt = w->push_cnt;
    hp.halo_e = w->halo_e;
    hp.own = dp<Snap<T>>(w->snap[c % 2], 0);
    hp.peer_mail = reinterpret_cast<char *const *>(w->peer_flags_dev);
    hp.mail = reinterpret_cast<const char *>(w->flags);
    hp.lay = MailLayout::make(w->P, w->S, w->esz, w->boxes);
    hp.epoch = w->epoch;
    hp.rank = (int32_t)w->rank;
    hp.P = (int32_t)w->P;
    hp.n_local = w->n_local;
    hp.lo = w->lo;
    hp.S = w->S;
    hp.timeout_ticks = 500000000;      // 5 s at 100 MHz
    hp.quat = w->boxes ? dp<T>(w->qsnap[nsp], 0) : nullptr;
    return hp;
}

// in-place all-gather of the snapshot of parity sp (and, box worlds, of the
// orientation snapshot: [P][S][4] the same way)
int rccl_gather(rb_world *w, int sp, hipStream_t s) {
    const size_t n = (size_t)4 * w->S;
    const ncclDataType_t ty = w->dtype == RB_F64 ? ncclFloat64 : ncclFloat32;
    for (int k = 0; k < (w->boxes ? 2 : 1); ++k) {
        char *buf = static_cast<char *>(k == 0 ? w->snap[sp] : w->qsnap[sp]);
        const ncclResult_t r = rccl().AllGather(buf + (size_t)w->esz * n * w->rank, buf, n, ty, w->comm, s);
        if (r != ncclSuccess) return fail(RB_ENODEV, "ncclAllGather: %s", rccl().GetErrorString(r));
    }
    return RB_OK;
}

// The in-library exchange after the step kernel of step c (which put the own
// bodies' new positions in this rank's slice of the next snapshot): the
// in-place all-gather of that snapshot, then the insert of every other
// rank's bodies into the next table (as rb_shard_exchange_done).
int shard_exchange(rb_world *w, hipStream_t s, int64_t c) {
    const int nsp = 1 - (int)(c % 2);
    if (w->p2p && w->halo) {
        const hipError_t he = w->dtype == RB_F64 ? launch_halo_exchange<double>(make_halo<double>(w, c, nsp), s)
                                                 : launch_halo_exchange<float>(make_halo<float>(w, c, nsp), s);
        HIPCHK(he);
        return RB_OK;
    }
    if (w->p2p) {
        hipError_t pe;
        if (w->dtype == RB_F64) {
            P2PParams<double> pp = make_p2p<double>(w, c, nsp);
            pe = launch_p2p_exchange<double>(pp, s);
        } else {
            P2PParams<float> pp = make_p2p<float>(w, c, nsp);
            pe = launch_p2p_exchange<float>(pp, s);
        }
        HIPCHK(pe);
        return RB_OK;
    }
    if (int rc = rccl_gather(w, nsp, s)) return rc;
    const hipError_t ie =
        w->dtype == RB_F64
            ? launch_insert<double>(make_insert<double>(w, nsp, 0, w->N, w->lo, w->lo + w->n_local), s)
            : launch_insert<float>(make_insert<float>(w, nsp, 0, w->N, w->lo, w->lo + w->n_local), s);
    HIPCHK(ie);
    return RB_OK;
}
// one sharded step: step kernel, then the exchange
int shard_one(rb_world *w, hipStream_t s, int64_t c, double dt, double e, double mu, double thr) {
    const int rc = launch_one(w, s, c, dt, e, mu, thr);
    return rc ? rc : shard_exchange(w, s, c);
}

void drop_graphs(rb_world *w) {
    for (auto &kv : w->graphs) (void)hipGraphExecDestroy(kv.second.ex);
    w->graphs.clear();
}

constexpr size_t GRAPH_CACHE_MAX = 32;

// evict least recently used graphs until `room` more fit
void evict_graphs(rb_world *w, size_t room) {
    while (!w->graphs.empty() && w->graphs.size() + room > GRAPH_CACHE_MAX) {
        auto lru = w->graphs.begin();
        for (auto it = w->graphs.begin(); it != w->graphs.end(); ++it)
            if (it->second.used < lru->second.used) lru = it;
        (void)hipGraphExecDestroy(lru->second.ex);
        w->graphs.erase(lru);
    }
}

// Table generations are 32-bit and only grow: before they would wrap (after
// ~4e9 steps of one world) the bucket lines are zeroed and the table
// rebuilt at generation 2 — from the snapshot, which holds every body's
// position except in a halo-exchanging shard (there: an error).
int gen_guard(rb_world *w, int64_t nsteps) {
    const uint64_t g = (uint32_t)(w->gen_off + (uint32_t)w->c);
    if (g + (uint64_t)nsteps + 4 < (1ull << 32)) return RB_OK;
    if (w->halo)
        return fail(RB_EOVERFLOW, "table generations exhausted after ~4e9 steps of a halo-exchanging shard: "
                                  "the sharded world must be recreated");
    HIPCHK(hipStreamSynchronize(w->stream));
    for (int k = 0; k < 2; ++k) {
        WCHK(wfill(w, w->ids[k], 0, sizeof(uint32_t) * LINE_WORDS * w->H));
        WCHK(wfill(w, w->spill[k], 0, sizeof(uint32_t) * SPILL_LINE_WORDS * SPILL_LINES));
    }
    w->gen_off = 1u - (uint32_t)w->c;   // prime() makes step c's generation 2
    w->primed = false;
    return RB_OK;
}

int enqueue_steps(rb_world *w, int64_t nsteps, double dt, double e, double mu, double thr, bool sharded = false);

// every run that awaits its check at the next sync point (tile runs)
int tile_finish(rb_world *w);
int finish_pending(rb_world *w) { return tile_finish(w); }

// Guarded chunks (enqueue_steps): the chunk-start copy (state rows,
// snapshot, box orientations, error word), the check after the chunk (error
// word, deferral counts: one host sync), the roll-back.
constexpr int64_t GUARD_MIN_STEPS = 64;   // shorter synchronous calls are not guarded (their
                                          // save + check would cost a few % of the call)
size_t chunk_save_bytes(const rb_world *w) {
    return (size_t)w->esz * (13 * (size_t)w->S + 8 * (size_t)w->Npad) + sizeof(int32_t);
}
int chunk_save(rb_world *w) {
    if (!w->opt_save) {
        HIPCHK(hipMalloc(&w->opt_save, chunk_save_bytes(w)));
        HIPCHK(hipHostMalloc((void **)&w->defer_host, sizeof(int32_t) * 4, 0));
    }
    char *o = static_cast<char *>(w->opt_save);
    const size_t st = (size_t)w->esz * 13 * w->S, sn = (size_t)w->esz * 4 * w->Npad;
    HIPCHK(hipMemcpyAsync(o, w->state, st, hipMemcpyDeviceToDevice, w->stream));
    HIPCHK(hipMemcpyAsync(o + st, w->snap[w->sp()], sn, hipMemcpyDeviceToDevice, w->stream));
    if (w->boxes) HIPCHK(hipMemcpyAsync(o + st + sn, w->qsnap[w->sp()], sn, hipMemcpyDeviceToDevice, w->stream));
    HIPCHK(hipMemcpyAsync(o + st + 2 * sn, w->err, sizeof(int32_t), hipMemcpyDeviceToDevice, w->stream));
    // the error bits from before the chunk (an earlier rb_step_async), read with the check
    HIPCHK(hipMemcpyAsync(w->defer_host + 3, w->err, sizeof(int32_t), hipMemcpyDeviceToHost, w->stream));
    if (w->boxes) HIPCHK(hipMemsetAsync(w->defer_cnt, 0, sizeof(int32_t) * 2, w->stream));
    return RB_OK;
}
int chunk_check(rb_world *w, int32_t &err, bool &deferred) {
    HIPCHK(hipMemcpyAsync(w->defer_host, w->err, sizeof(int32_t), hipMemcpyDeviceToHost, w->stream));
    if (w->boxes) HIPCHK(hipMemcpyAsync(w->defer_host + 1, w->defer_cnt, sizeof(int32_t) * 2, hipMemcpyDeviceToHost, w->stream));
    HIPCHK(hipStreamSynchronize(w->stream));
    err = w->defer_host[0] & ~w->defer_host[3];       // raised during this chunk
    if (w->diag_overflow > 0) { --w->diag_overflow; err |= ERR_BUCKET_OVERFLOW; }
    deferred = w->boxes && (w->defer_host[1] | w->defer_host[2]) != 0;
    return RB_OK;
}
int chunk_restore(rb_world *w) {
    const char *o = static_cast<const char *>(w->opt_save);
    const size_t st = (size_t)w->esz * 13 * w->S, sn = (size_t)w->esz * 4 * w->Npad;
    HIPCHK(hipMemcpyAsync(w->state, o, st, hipMemcpyDeviceToDevice, w->stream));
    HIPCHK(hipMemcpyAsync(w->snap[w->sp()], o + st, sn, hipMemcpyDeviceToDevice, w->stream));
    if (w->boxes) HIPCHK(hipMemcpyAsync(w->qsnap[w->sp()], o + st + sn, sn, hipMemcpyDeviceToDevice, w->stream));
    w->err_pub = false;
    HIPCHK(hipMemcpyAsync(w->err, o + st + 2 * sn, sizeof(int32_t), hipMemcpyDeviceToDevice, w->stream));
    if (w->boxes) HIPCHK(hipMemsetAsync(w->defer_cnt, 0, sizeof(int32_t) * 2, w->stream));
    w->primed = false;
    w->tile_valid_sp = -1;
    return RB_OK;
}
// twice the buckets (both tables, emptied), if under the world's limit; the
// linear layout's period gets the extra bit (refit_from_device re-splits it)
int grow_table(rb_world *w, bool &grown) {
    grown = false;
    if (w->H * 2 > w->hmax) return RB_OK;
    HIPCHK(hipStreamSynchronize(w->stream));
    drop_graphs(w);                                   // H and the grid are captured kernel arguments
    const int64_t H = w->H * 2;
    for (int k = 0; k < 2; ++k) {
        HIPCHK(hipFree(w->ids[k]));
        w->ids[k] = nullptr;
        HIPCHK(hipMalloc((void **)&w->ids[k], sizeof(uint32_t) * LINE_WORDS * H));
        WCHK(wfill(w, w->ids[k], 0, sizeof(uint32_t) * LINE_WORDS * H));
        if (w->pos[k]) {
            HIPCHK(hipFree(w->pos[k]));
            w->pos[k] = nullptr;
            HIPCHK(hipMalloc(&w->pos[k], (size_t)w->esz * 4 * LINE_WORDS * H));
        }
    }
    w->H = H;
    if ((w->group >> 24) & 1) {
        const int lx = (w->group >> 12) & 15, ly = (w->group >> 16) & 15;
        w->group += lx < 15 ? (1 << 12) : ly < 15 ? (1 << 16) : (1 << 20);
    }
    w->fit_valid = false;
    w->primed = false;
    w->table_grows += 1;
    grown = true;
    return RB_OK;
}

// max_partners raised to 32 (the second kernel instantiation), contact
// records resized to match
int grow_partners(rb_world *w) {
    HIPCHK(hipStreamSynchronize(w->stream));
    drop_graphs(w);                                   // the instantiation is chosen at capture
    w->maxp = 32;
    w->maxrec = 4 * w->n_planes + (w->boxes ? 4 : 1) * w->maxp;
    if (w->rec_count) {
        const size_t slots = (size_t)w->maxrec * (w->S > 0 ? w->S : 1);
        void *old[] = {w->rec_partner, w->rec_kind, w->rec_dist};
        for (void *b : old) HIPCHK(hipFree(b));
        w->rec_partner = nullptr; w->rec_kind = nullptr; w->rec_dist = nullptr;
        HIPCHK(hipMalloc((void **)&w->rec_partner, sizeof(int32_t) * slots));
        HIPCHK(hipMalloc((void **)&w->rec_kind, sizeof(int32_t) * slots));
        HIPCHK(hipMalloc(&w->rec_dist, (size_t)w->esz * slots));
    }
    w->partner_grows += 1;
    return RB_OK;
}

// the layout period refitted to the current positions (the snapshot)
int refit_from_device(rb_world *w) {
    std::vector<double> q((size_t)7 * w->N, 0.0);
    if (w->dtype == RB_F64) {
        std::vector<double> sn((size_t)4 * w->N);
        HIPCHK(hipMemcpyAsync(sn.data(), w->snap[w->sp()], sizeof(double) * sn.size(), hipMemcpyDeviceToHost, w->stream));
        HIPCHK(hipStreamSynchronize(w->stream));
        for (int64_t b = 0; b < w->N; ++b)
            for (int d = 0; d < 3; ++d) q[(size_t)(7 * b + d)] = sn[(size_t)(4 * b + d)];
    } else {
        std::vector<float> sn((size_t)4 * w->N);
        HIPCHK(hipMemcpyAsync(sn.data(), w->snap[w->sp()], sizeof(float) * sn.size(), hipMemcpyDeviceToHost, w->stream));
        HIPCHK(hipStreamSynchronize(w->stream));
        for (int64_t b = 0; b < w->N; ++b)
            for (int d = 0; d < 3; ++d) q[(size_t)(7 * b + d)] = sn[(size_t)(4 * b + d)];
    }
    fit_period(w, q.data(), true);
    return RB_OK;
}


// ---- captured step graphs ---------------------------------------------------
// A sequence of launches covering K steps from step c0 (`seq(stream, c0)`),
// captured once per start parity and replayed (rb_world::graphs, keyed by the
// step count, parity, step parameters and variant).
int graph_replay(rb_world *w, int64_t K, int variant, double dt, double e, double mu, double thr,
                 const std::function<int(hipStream_t, int64_t)> &seq) {
    const bool tile_graph = (variant & 16) && w->tile_pub_host_d;   // (a tile run's: its words too)
    auto key = std::make_tuple(K, (int)(w->c % 2), dt, e, mu, thr, variant);
    auto it = w->graphs.find(key);
    if (it == w->graphs.end()) {
        evict_graphs(w, 2);
        // capture both parities at once, so later calls starting at either
        // replay without a capture (a parity still cached is kept; both
        // entries get the current tick, so the one not launched now is not
        // the first evicted).  No other thread inside the library meanwhile
        // (CaptureScope).
        CaptureScope capture_scope_;
        for (int c0 = 0; c0 < 2; ++c0) {
            const auto k0 = std::make_tuple(K, c0, dt, e, mu, thr, variant);
            auto old = w->graphs.find(k0);
            if (old != w->graphs.end()) { old->second.used = w->graph_tick; continue; }
            hipGraph_t graph;
            hipGraphExec_t ex;
            HIPCHK(hipStreamBeginCapture(w->cap_stream, hipStreamCaptureModeThreadLocal));
            int rc = seq(w->cap_stream, c0);
            const hipError_t pe = rc ? hipSuccess
                                     : tile_graph ? launch_publish_err(w->err, w->err_host_d, w->cap_stream, w->tile_why,
                                                                       w->tile_commits, w->tile_pub_host_d)
                                                  : launch_publish_err(w->err, w->err_host_d, w->cap_stream);
            if (rc || pe != hipSuccess) {
                (void)hipStreamEndCapture(w->cap_stream, &graph);
                if (rc) return rc;
                HIPCHK(pe);
            }
            HIPCHK(hipStreamEndCapture(w->cap_stream, &graph));
            HIPCHK(hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0));
            (void)hipGraphDestroy(graph);
            w->graphs[k0] = rb_world::GraphEntry{ex, w->graph_tick};
        }
        it = w->graphs.find(key);
    }
    it->second.used = ++w->graph_tick;
    HIPCHK(hipGraphLaunch(it->second.ex, w->stream));
    w->err_pub = true;                               // (the graph ends in publish_err_kernel)
    w->tile_pub = tile_graph;
    return RB_OK;
}

// The period-split scoring shared by fit_period (the world's tables) and
// xb_fit_cuts (the blocks' tables): group keys packed 21 bits per axis.
constexpr int64_t PERIOD_OFF = 1 << 20;                  // group coordinates kept in [-2^20, 2^20)
inline int64_t period_pack(int64_t gx, int64_t gy, int64_t gz) {
    return ((gx + PERIOD_OFF) << 42) | ((gy + PERIOD_OFF) << 21) | (gz + PERIOD_OFF);
}
inline int64_t period_unpack(int64_t k, int d) { return ((k >> (42 - 21 * d)) & ((1 << 21) - 1)) - PERIOD_OFF; }
// The groups a search reads (the occupied ones, sorted unique, and their
// neighbours; above 8,192 occupied groups the occupied ones alone), with
// their coordinates and an occupied flag.
struct PeriodSet {
    std::vector<int64_t> qg[3];
    std::vector<uint8_t> qocc;
    explicit PeriodSet(std::vector<int64_t> occ) {
        std::sort(occ.begin(), occ.end());
        occ.erase(std::unique(occ.begin(), occ.end()), occ.end());
        std::vector<int64_t> q;
        q.reserve(occ.size() * 27);
        if (occ.size() > 8192) q = occ;
        else for (int64_t k : occ)
            for (int dz = -1; dz <= 1; ++dz)
                for (int dy = -1; dy <= 1; ++dy)
                    for (int dx = -1; dx <= 1; ++dx)
                        q.push_back(period_pack(period_unpack(k, 0) + dx, period_unpack(k, 1) + dy, period_unpack(k, 2) + dz));
        std::sort(q.begin(), q.end());
        q.erase(std::unique(q.begin(), q.end()), q.end());
        qocc.resize(q.size());
        for (int d = 0; d < 3; ++d) qg[d].resize(q.size());
        for (size_t t = 0; t < q.size(); ++t) {
            for (int d = 0; d < 3; ++d) qg[d][t] = period_unpack(q[t], d);
            qocc[t] = std::binary_search(occ.begin(), occ.end(), q[t]) ? 1 : 0;
        }
    }
    // groups a search reads that share a run of buckets with another group,
    // at least one of them occupied, under the period 2^l[0] x 2^l[1] x 2^l[2]
    int64_t collisions(const int l[3], std::vector<uint64_t> &f) const {
        f.resize(qocc.size());
        for (size_t t = 0; t < qocc.size(); ++t) {
            uint64_t idx = 0;
            int sh = 0;
            for (int d = 0; d < 3; ++d) {
                idx |= ((uint64_t)qg[d][t] & ((1ull << l[d]) - 1)) << sh;
                sh += l[d];
            }
            f[t] = (idx << 1) | qocc[t];
        }
        std::sort(f.begin(), f.end());
        int64_t coll = 0;
        for (size_t a = 0; a < f.size();) {
            size_t e = a;
            bool any_occ = false;
            while (e < f.size() && (f[e] >> 1) == (f[a] >> 1)) any_occ |= (f[e++] & 1);
            if (any_occ) coll += (int64_t)(e - a) - 1;
            a = e;
        }
        return coll;
    }
};
// The split of lg period bits with the fewest collisions summed over the
// sets; ties: fewest axes the period does not cover (need[d]: groups of
// extent per axis), then the most even cover.
inline void best_period_split(const std::vector<PeriodSet> &sets, const double need[3], int lg, int best[3]) {
    std::vector<uint64_t> f;
    int64_t best_c = -1;
    int best_nf = 0;
    double best_fold = 0.0;
    for (int lx = 0; lx <= lg && lx <= 15; ++lx)
        for (int ly = 0; lx + ly <= lg && ly <= 15; ++ly) {
            const int lz = lg - lx - ly;
            if (lz > 15) continue;
            const int l[3] = {lx, ly, lz};
            int64_t coll = 0;
            for (const PeriodSet &ps : sets) coll += ps.collisions(l, f);
            double fold = 0.0;
            int nf = 0;                                  // axes the period does not cover
            for (int d = 0; d < 3; ++d) {
                fold = std::max(fold, need[d] / double(1 << l[d]));
                nf += need[d] > double(1 << l[d]);
            }
            if (best_c < 0 || coll < best_c || (coll == best_c && nf < best_nf) ||
                (coll == best_c && nf == best_nf && fold < best_fold - 1e-12)) {
                best_c = coll;
                best_nf = nf;
                best_fold = fold;
                best[0] = lx; best[1] = ly; best[2] = lz;
            }
        }
}

// ---- the cell-ordered tile form (rb_tiles.hip) -----------------
bool tile_eligible(const rb_world *w) {
    if (w->tile_mode == 0 || w->tile_replaying || w->P != 1 || !w->all_spheres || w->law != RB_LAW_MUJOCO || w->xfrc || w->timing)
        return false;
    // (more than TILE_TYPES distinct (m, I): the hashed forms, which read them by id)
    if (w->maxp > 32 || w->n_local <= 0 || w->N > (int64_t)TILE_ID_MASK + 1 || w->tile_ntypes < 1) return false;
    return w->tile_mode == 1 || w->n_local >= w->tile_min_bodies;
}

// The tile grid from body positions (x, y at pos[k * stride], pos[k * stride + 1]):
// columns of the hashed cell size; tc columns per tile edge so that a tile
// holds ~80 bodies on average (a slot steps at most TILE_THREADS) and none
// holds more than 7/8 of that limit at the fit; ntx x nty slots covering the
// scene's extent plus a margin (periodic: a scene that outgrows it folds
// onto itself, which stays exact).
void tile_fit(rb_world *w, const double *pos, int64_t stride) {
    const double inv = w->inv_cs;
    std::vector<int64_t> cols;
    cols.reserve((size_t)w->N);
    int64_t lo[2] = {INT64_MAX, INT64_MAX}, hi[2] = {INT64_MIN, INT64_MIN};
    for (int64_t b = 0; b < w->N; ++b) {
        const double fx = pos[b * stride] * inv, fy = pos[b * stride + 1] * inv;
        if (!(fabs(fx) < 1e9 && fabs(fy) < 1e9)) continue;
        const int64_t cx = (int64_t)floor(fx), cy = (int64_t)floor(fy);
        lo[0] = std::min(lo[0], cx); hi[0] = std::max(hi[0], cx);
        lo[1] = std::min(lo[1], cy); hi[1] = std::max(hi[1], cy);
        cols.push_back(((cx + (1 << 30)) << 31) | (cy + (1 << 30)));
    }
    if (cols.empty()) { lo[0] = lo[1] = 0; hi[0] = hi[1] = 0; }
    std::sort(cols.begin(), cols.end());
    const int64_t nocc = std::max<int64_t>(1, (int64_t)(std::unique(cols.begin(), cols.end()) - cols.begin()));
    const double per_col = (double)std::max<int64_t>(1, (int64_t)cols.size()) / (double)nocc;
    int tc = (int)lround(sqrt(80.0 / per_col));
    tc = std::max(TILE_TC_MIN, std::min(TILE_TC_MAX, tc));
    if (const char *ev = getenv("RBHIP_TILE_COLS")) tc = std::max(TILE_TC_MIN, std::min(TILE_TC_MAX, atoi(ev)));
    // the densest tile at this fit under 3/4 of a slot's limit
    for (; tc > TILE_TC_MIN; --tc) {
        std::vector<int64_t> t;
        t.reserve(cols.size());
        for (int64_t b = 0; b < w->N; ++b) {
            const double fx = pos[b * stride] * inv, fy = pos[b * stride + 1] * inv;
            if (!(fabs(fx) < 1e9 && fabs(fy) < 1e9)) continue;
            const int64_t tx = (int64_t)floor(floor(fx) / tc), ty = (int64_t)floor(floor(fy) / tc);
            t.push_back(((tx + (1 << 30)) << 31) | (ty + (1 << 30)));
        }
        std::sort(t.begin(), t.end());
        int64_t worst = 0;
        for (size_t a = 0; a < t.size();) {
            size_t e = a;
            while (e < t.size() && t[e] == t[a]) ++e;
            worst = std::max<int64_t>(worst, (int64_t)(e - a));
            a = e;
        }
        if (worst <= 7 * TILE_THREADS / 8) break;
    }
    int64_t ntx = (hi[0] - lo[0]) / tc + 3, nty = (hi[1] - lo[1]) / tc + 3;
    // a scene spread far (outliers): fold instead of launching empty slots
    const int64_t max_slots = 4 * ((w->N + 23) / 24) + 64;
    while (ntx * nty > max_slots) {
        if (ntx >= nty) ntx = (ntx + 1) / 2; else nty = (nty + 1) / 2;
    }
    w->tile_tc = tc;
    w->tile_ntx = (int32_t)std::max<int64_t>(3, ntx);
    w->tile_nty = (int32_t)std::max<int64_t>(3, nty);
    w->tile_fit_valid = true;
}

size_t tile_bins_bytes(const rb_world *w) {
    const size_t slots = (size_t)w->tile_ntx * w->tile_nty, cap = (size_t)w->tile_cap, esz = (size_t)w->esz;
    return slots * TILE_OFFW * 4 + slots * cap * (4 * esz + 4 + TILE_STW * esz) + 256 +
           (size_t)TILE_FARMAX * (4 * esz + 4 + TILE_STW * esz) + 256;
}
template <typename T> TileBins<T> tile_bins(const rb_world *w, int sp) {
    const size_t slots = (size_t)w->tile_ntx * w->tile_nty, cap = (size_t)w->tile_cap;
    char *b = static_cast<char *>(w->tile_mem) + (size_t)sp * tile_bins_bytes(w);
    TileBins<T> t;
    t.off = reinterpret_cast<int32_t *>(b);
    b += slots * TILE_OFFW * 4;
    t.pos = reinterpret_cast<Snap<T> *>(b);
    b += slots * cap * 4 * sizeof(T);
    t.st = reinterpret_cast<T *>(b);
    b += slots * cap * TILE_STW * sizeof(T);
    t.id = reinterpret_cast<int32_t *>(b);
    b += (slots * cap * 4 + 255) / 256 * 256;
    t.far_hdr = reinterpret_cast<unsigned long long *>(b);
    b += 256;
    t.far_pos = reinterpret_cast<Snap<T> *>(b);
    b += (size_t)TILE_FARMAX * 4 * sizeof(T);
    t.far_st = reinterpret_cast<T *>(b);
    b += (size_t)TILE_FARMAX * TILE_STW * sizeof(T);
    t.far_id = reinterpret_cast<int32_t *>(b);
    return t;
}

// tile_build / tile_alloc: the auto mode's bins would not fit (a scene spread
// far, folded onto many mostly empty slots, or device memory short): the
// world steps hashed from now on
constexpr int TILE_DECLINED = 1;
constexpr size_t TILE_AUTO_MAX_BYTES_PER_BODY = 2048;   // flat scenes need ~0.4 KB

// the words the pending tile runs' checks read
int tile_alloc_words(rb_world *w) {
    if (w->tile_gen) return RB_OK;
    HIPCHK(hipMalloc((void **)&w->tile_gen, 2 * sizeof(uint32_t)));
    HIPCHK(hipMalloc((void **)&w->tile_why, sizeof(int32_t)));
    HIPCHK(hipMalloc((void **)&w->tile_commits, sizeof(unsigned long long)));
    WCHK(wfill(w, w->tile_why, 0, sizeof(int32_t)));
    WCHK(wfill(w, w->tile_commits, 0, sizeof(unsigned long long)));
    HIPCHK(hipHostMalloc((void **)&w->tile_host, 4 * sizeof(int64_t), 0));
    HIPCHK(hipHostMalloc((void **)&w->tile_pub_host, 2 * sizeof(int64_t), hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer((void **)&w->tile_pub_host_d, w->tile_pub_host, 0));
    w->tile_commits_seen = 0;
    return RB_OK;
}

// Auto mode retires the tile form (a roll-back, or bins it will not
// allocate): the bins go too (hundreds of MB at millions of bodies), and the
// graphs that captured their pointers
int tile_retire(rb_world *w) {
    w->tile_mode = 0;
    w->tile_valid_sp = -1;
    if (!w->tile_mem && !w->tile_fill) return RB_OK;
    HIPCHK(hipStreamSynchronize(w->stream));
    drop_graphs(w);
    if (w->tile_mem) HIPCHK(hipFree(w->tile_mem));
    if (w->tile_fill) HIPCHK(hipFree(w->tile_fill));
    w->tile_mem = nullptr;
    w->tile_fill = nullptr;
    w->tile_mem_bytes = 0;
    return RB_OK;
}

int tile_alloc(rb_world *w) {
    const size_t need = 2 * tile_bins_bytes(w);
    const size_t slots = (size_t)w->tile_ntx * w->tile_nty;
    if (w->tile_mem && w->tile_mem_bytes >= need && w->tile_fill) {
        // the fill scratch is sized for the slots too
        return RB_OK;
    }
    if (w->tile_mode == -1 && need > TILE_AUTO_MAX_BYTES_PER_BODY * (size_t)w->N) {
        if (int rc = tile_retire(w)) return rc;
        return TILE_DECLINED;
    }
    HIPCHK(hipStreamSynchronize(w->stream));
    drop_graphs(w);                                  // captured bin pointers
    if (w->tile_mem) { HIPCHK(hipFree(w->tile_mem)); w->tile_mem = nullptr; }
    if (w->tile_fill) { HIPCHK(hipFree(w->tile_fill)); w->tile_fill = nullptr; }
    if (hipMalloc(&w->tile_mem, need) != hipSuccess ||
        hipMalloc((void **)&w->tile_fill, slots * TILE_OFFW * 4) != hipSuccess) {
        (void)hipGetLastError();
        if (w->tile_mem) (void)hipFree(w->tile_mem);
        w->tile_mem = nullptr;
        w->tile_mem_bytes = 0;
        if (w->tile_mode == -1) {
            if (int rc = tile_retire(w)) return rc;
            return TILE_DECLINED;
        }
        return fail(RB_ENOMEM, "tile bins: hipMalloc of %zu bytes failed", need);
    }
    w->tile_mem_bytes = need;
    return tile_alloc_words(w);
}

template <typename T> TileIO<T> make_tile_io(rb_world *w, int64_t c) {
    w->err_pub = false;
    TileIO<T> p{};
    const int sp = (int)(c % 2);
    p.bins = tile_bins<T>(w, sp);
    p.gen = w->tile_gen + sp;
    p.snap = dp<Snap<T>>(w->snap[sp], 0);
    p.st = BodyState<T>{dp<T>(w->state, 0), w->S};
    p.fill = w->tile_fill;
    p.type_of = w->tile_type_of;
    p.tc = w->tile_tc; p.ntx = w->tile_ntx; p.nty = w->tile_nty; p.cap = w->tile_cap;
    p.inv_col = (T)w->inv_cs;
    p.n = w->N;
    p.err = w->err;
    p.why = w->tile_why;
    p.commits = w->tile_commits;
    return p;
}

template <typename T> TileParams<T> make_tile_step(rb_world *w, int64_t c, double dt, double e, double mu, double thr) {
    w->err_pub = false;
    TileParams<T> p{};
    const int sp = (int)(c % 2);
    p.cur = tile_bins<T>(w, sp);
    p.next = tile_bins<T>(w, 1 - sp);
    p.gen_cur = w->tile_gen + sp;
    p.gen_next = w->tile_gen + (1 - sp);
    p.sp = make_step<T>(w, c, dt, e, mu, thr, false);
    p.ntypes = w->tile_ntypes;
    for (int t = 0; t < w->tile_ntypes; ++t)
        for (int k = 0; k < 4; ++k) p.types[t][k] = (T)w->tile_type_val[t][k];
    p.tc = w->tile_tc; p.ntx = w->tile_ntx; p.nty = w->tile_nty; p.cap = w->tile_cap;
    p.inv_col = (T)w->inv_cs;
    p.why = w->tile_why;
    return p;
}

// the bins of step c from the id-ordered state (snapshot and state rows)
int tile_build(rb_world *w) {
    if (!w->tile_fit_valid) {
        // positions: the staging when it mirrors the state, else the snapshot
        if (w->io_q_h && w->mirror_version == w->state_version) {
            tile_fit(w, w->io_q_h, 7);
        } else {
            std::vector<double> q((size_t)4 * w->N);
            if (w->dtype == RB_F64) {
                HIPCHK(hipMemcpyAsync(q.data(), w->snap[w->sp()], sizeof(double) * q.size(), hipMemcpyDeviceToHost, w->stream));
                HIPCHK(hipStreamSynchronize(w->stream));
            } else {
                std::vector<float> f(q.size());
                HIPCHK(hipMemcpyAsync(f.data(), w->snap[w->sp()], sizeof(float) * f.size(), hipMemcpyDeviceToHost, w->stream));
                HIPCHK(hipStreamSynchronize(w->stream));
                for (size_t k = 0; k < f.size(); ++k) q[k] = f[k];
            }
            tile_fit(w, q.data(), 4);
        }
        drop_graphs(w);                              // the grid is a captured kernel argument
    }
    if (int rc = tile_alloc(w)) return rc;
    const int sp = w->sp();
    const size_t slots = (size_t)w->tile_ntx * w->tile_nty;
    HIPCHK(hipMemsetAsync(w->tile_fill, 0, slots * TILE_OFFW * 4, w->stream));
    for (int k = 0; k < 2; ++k) {
        // far lists empty (tag 0: never a live generation)
        HIPCHK(hipMemsetAsync(w->dtype == RB_F64 ? (void *)tile_bins<double>(w, k).far_hdr : (void *)tile_bins<float>(w, k).far_hdr,
                              0, sizeof(unsigned long long), w->stream));
    }
    HIPCHK(hipMemsetAsync(w->dtype == RB_F64 ? (void *)tile_bins<double>(w, sp).off : (void *)tile_bins<float>(w, sp).off, 0,
                          slots * TILE_OFFW * 4, w->stream));
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)(w->tile_gen + sp), 1, 1, w->stream));
    HIPCHK(w->dtype == RB_F64 ? launch_tile_build<double>(make_tile_io<double>(w, w->c), w->stream)
                              : launch_tile_build<float>(make_tile_io<float>(w, w->c), w->stream));
    w->tile_valid_sp = sp;
    w->tile_stats[3] += 1;
    return RB_OK;
}

// One run of n tile steps from step c (graph-replayed in chunks; the last
// chunk ends with the unbin kernel), recorded as pending until checked.
int tile_run(rb_world *w, int64_t n, double dt, double e, double mu, double thr) {
    if (w->tile_valid_sp != w->sp()) {
        if (int rc = finish_pending(w)) return rc;  // (the build reads the id-ordered state)
        if (int rc = tile_build(w)) return rc;
    }
    const bool f64 = w->dtype == RB_F64;
    const int64_t c0 = w->c, chunk_max = 512;
    int64_t left = n;
    while (left > 0) {
        const int64_t K = left > chunk_max ? chunk_max : left;
        const bool last = K == left;
        const int variant = 16 | (int)w->record | (last ? 32 : 0);
        int rc = graph_replay(w, K, variant, dt, e, mu, thr, [&](hipStream_t s, int64_t cs) {
            for (int64_t k = 0; k < K; ++k) {
                const hipError_t r = f64 ? launch_tile_step<double>(make_tile_step<double>(w, cs + k, dt, e, mu, thr), w->maxp, s)
                                         : launch_tile_step<float>(make_tile_step<float>(w, cs + k, dt, e, mu, thr), w->maxp, s);
                HIPCHK(r);
            }
            if (last) HIPCHK(f64 ? launch_tile_unbin<double>(make_tile_io<double>(w, cs + K), s)
                                 : launch_tile_unbin<float>(make_tile_io<float>(w, cs + K), s));
            return (int)RB_OK;
        });
        if (rc) return rc;
        w->c += K;
        left -= K;
    }
    w->tile_valid_sp = w->sp();
    w->primed = false;                               // the hashed forms' table is stale
    w->tile_pending.push_back(rb_world::TileRun{c0, n, dt, e, mu, thr});
    w->tile_stats[0] += 1;
    return RB_OK;
}

// The check of the pending tile runs: every run whose unbin committed is
// done; the first run that raised ERR_TILE and every run after it are
// replayed, from the id-ordered state (which still holds that run's start),
// by the hashed-cell forms — which report any real error themselves.
int tile_finish(rb_world *w) {
    if (w->tile_pending.empty()) return RB_OK;
    int32_t err, why;
    unsigned long long commits;
    if (w->err_pub && w->tile_pub) {
        // the last tile graph published the three words (publish_err_kernel)
        HIPCHK(hipStreamSynchronize(w->stream));
        err = __atomic_load_n(w->err_host, __ATOMIC_ACQUIRE);
        why = (int32_t)__atomic_load_n(w->tile_pub_host, __ATOMIC_ACQUIRE);
        commits = (unsigned long long)__atomic_load_n(w->tile_pub_host + 1, __ATOMIC_ACQUIRE);
    } else {
        HIPCHK(hipMemcpyAsync(w->tile_host, w->err, sizeof(int32_t), hipMemcpyDeviceToHost, w->stream));
        HIPCHK(hipMemcpyAsync(w->tile_host + 1, w->tile_why, sizeof(int32_t), hipMemcpyDeviceToHost, w->stream));
        HIPCHK(hipMemcpyAsync(w->tile_host + 2, w->tile_commits, sizeof(unsigned long long), hipMemcpyDeviceToHost, w->stream));
        HIPCHK(hipStreamSynchronize(w->stream));
        err = (int32_t)reinterpret_cast<int32_t *>(w->tile_host)[0];
        why = (int32_t)reinterpret_cast<int32_t *>(w->tile_host + 1)[0];
        commits = (unsigned long long)w->tile_host[2];
    }
    const size_t ok = (size_t)(commits - w->tile_commits_seen);
    w->tile_commits_seen = commits;
    std::vector<rb_world::TileRun> runs;
    runs.swap(w->tile_pending);
    for (size_t k = 0; k < ok && k < runs.size(); ++k) w->tile_stats[1] += runs[k].n;
    if (!(err & ERR_TILE)) {
        if (w->tile_backoff > 0) w->tile_backoff /= 2;
        return RB_OK;
    }
    // roll back to the start of the first failed run and replay it and
    // every later one with the hashed-cell forms (guarded chunks: the
    // replay grows max_partners or refits the table as a synchronous
    // rb_step would)
    const size_t first = std::min(ok, runs.size());
    const int32_t clean = err & ~ERR_TILE;
    w->err_pub = false;
    HIPCHK(hipMemcpyAsync(w->err, &clean, sizeof(int32_t), hipMemcpyHostToDevice, w->stream));
    HIPCHK(hipMemsetAsync(w->tile_why, 0, sizeof(int32_t), w->stream));
    HIPCHK(hipStreamSynchronize(w->stream));
    w->tile_valid_sp = -1;
    w->primed = false;
    w->tile_stats[2] += 1;
    w->tile_why_seen |= why;
    if (why & (TILE_WHY_CAP | TILE_WHY_WINDOW)) w->tile_fit_valid = false;   // the scene outgrew the fit
    w->tile_backoff = w->tile_backoff ? std::min(2 * w->tile_backoff, 64) : 1;
    w->tile_skip = w->tile_backoff;
    // auto mode: a scene that outgrew the tile slots once (pile-ups) tends to
    // keep doing so, and every retry costs a roll-back — step hashed from now on
    if (w->tile_mode == -1)
        if (int rc = tile_retire(w)) return rc;
    w->c = first < runs.size() ? runs[first].c0 : w->c;
    const bool saved = w->sync_call;
    w->sync_call = true;
    w->tile_replaying = true;
    int rc = RB_OK;
    for (size_t k = first; k < runs.size() && !rc; ++k) {
        const rb_world::TileRun &r = runs[k];
        rc = enqueue_steps(w, r.n, r.dt, r.e, r.mu, r.thr, false);
    }
    w->tile_replaying = false;
    w->sync_call = saved;
    return rc;
}

// nsteps steps (sharded: with the in-library exchange), graph-replayed
int enqueue_steps(rb_world *w, int64_t nsteps, double dt, double e, double mu, double thr, bool sharded) {
    if (nsteps < 0) return fail(RB_EINVAL, "nsteps < 0");
    if (!sharded && w->P != 1) return fail(RB_EINVAL, "rb_step on a sharded world: use rb_shard_run or rb_shard_step + exchange");
    if (sharded && !w->comm && !w->p2p) return fail(RB_EINVAL, "rb_shard_run before rb_shard_comm_init or rb_p2p_connect");
    if (sharded && w->law != RB_LAW_MUJOCO) return fail(RB_EUNSUPPORTED, "sharded stepping supports the default contact law only");
    if (!(dt > 0) || !(e >= 0) || !(mu >= 0) || !(thr >= 0))
        return fail(RB_EINVAL, "invalid step parameters dt=%g e=%g mu=%g thr=%g", dt, e, mu, thr);
    if (nsteps == 0) return RB_OK;
    HIPCHK(hipSetDevice(w->device));
    // the tile form for runs of >= 2 steps, or to continue from its bins;
    // pending tile runs chain (their check waits for the next sync point),
    // anything else first settles them
    const bool tile = !sharded && tile_eligible(w) && (nsteps >= 2 || w->tile_valid_sp == w->sp()) &&
                      w->tile_pending.size() < 256;
    if (tile && w->tile_skip > 0 && w->tile_valid_sp != w->sp()) {
        --w->tile_skip;                              // (back-off after a roll-back: this run steps hashed)
    } else if (tile) {
        w->state_version += 1;
        const int rc = tile_run(w, nsteps, dt, e, mu, thr);
        if (rc != TILE_DECLINED) return rc;          // (declined: the hashed forms below)
    }
    if (int rc = finish_pending(w)) return rc;
    w->state_version += 1;
    w->tile_valid_sp = -1;                           // the hashed forms advance the id-ordered state
    if (int rc = gen_guard(w, nsteps)) return rc;
    if (!w->primed || (w->law == RB_LAW_BALLS && (dt != w->prm_dt || e != w->prm_e || mu != w->prm_mu))) {
        int rc = prime(w, dt, e, mu);
        if (rc) return rc;
    }
    if (sharded && w->p2p && w->halo) {
        // the halo pushes of the run's first step test against the bounds of
        // the current positions (the insert kernels publish them after)
        const int nsp = w->sp();
        const hipError_t he = w->dtype == RB_F64 ? launch_halo_prime<double>(make_halo<double>(w, w->c, nsp), w->stream)
                                                 : launch_halo_prime<float>(make_halo<float>(w, w->c, nsp), w->stream);
        HIPCHK(he);
    }
    auto one = [&](hipStream_t s, int64_t c) {
        return sharded ? shard_one(w, s, c, dt, e, mu, thr) : launch_one(w, s, c, dt, e, mu, thr);
    };
    if (w->timing) {
        // eager launches, each step kernel bracketed by events on the launch stream
        for (int64_t k = 0; k < nsteps; ++k) {
            int rc = timed_launch(w, dt, e, mu, thr);
            if (!rc && sharded) rc = shard_exchange(w, w->stream, w->c);
            if (rc) return rc;
            ++w->c;
        }
        return RB_OK;
    }
    if (nsteps == 1) {
        int rc = one(w->stream, w->c);
        if (rc) return rc;
        ++w->c;
        return RB_OK;
    }
    // K > 1: replay a captured graph of K step nodes
    auto replay = [&](int64_t K, int variant) -> int {
        return graph_replay(w, K, variant, dt, e, mu, thr, [&](hipStream_t s, int64_t c0) {
            for (int64_t k = 0; k < K; ++k)
                if (int rc = one(s, c0 + k)) return rc;
            return (int)RB_OK;
        });
    };
    const int variant = (int)w->record | (sharded ? 2 : 0);
    const int64_t chunk_max = 512;
    int64_t left = nsteps;
    while (left > 0) {
        int64_t K = left > chunk_max ? chunk_max : left;
        bool opt = w->boxes && w->box_opt && !sharded && w->P == 1 && w->box_skip == 0;
        // a chunk run with the box kernel because of an earlier roll-back
        // counts down the back-off (guarded or not)
        const bool skipped = w->boxes && w->box_opt && !sharded && w->P == 1 && w->box_skip > 0;
        if (skipped) --w->box_skip;
        // a guarded chunk can be rolled back: optimistic box chunks, and long
        // chunks of a synchronous call (rb_step), whose broadphase layout is
        // refitted if the scene drifted out of it (a bucket overflowed)
        const bool guard = opt || (w->sync_call && K >= GUARD_MIN_STEPS && !sharded && w->P == 1 &&
                                   w->law == RB_LAW_MUJOCO);
        if (!guard) {
            if (int rc = replay(K, variant)) return rc;
            w->c += K;
            left -= K;
            continue;
        }
        bool refitted = false;
        for (;;) {
            if (int rc = chunk_save(w)) return rc;
            w->box_kernel_on = !opt;
            const int rc = replay(K, variant | (opt ? 4 : 0));
            w->box_kernel_on = true;
            if (rc) return rc;
            int32_t err = 0;
            bool deferred = false;
            if (int rc2 = chunk_check(w, err, deferred)) return rc2;
            if (opt) w->box_stats[0] += 1;
            // bucket overflow right after a fit of one step: a real overflow
            // (reported by the caller's error check)
            const bool overflow = (err & ERR_BUCKET_OVERFLOW) && !(refitted && K == 1);
            // more sphere partners than max_partners 16: the 32-partner kernels
            const bool partners = (err & ERR_PARTNER_OVERFLOW) && w->maxp < 32;
            deferred = deferred && opt;
            if (!overflow && !deferred && !partners) {
                if (opt && w->box_backoff > 0) w->box_backoff /= 2;
                break;
            }
            if (int rc3 = chunk_restore(w)) return rc3;
            if (deferred) {
                // a box-involved pair came into range: the chunk again, from
                // its start, with the box kernel; the next chunks keep it
                w->box_stats[1] += 1;
                w->box_backoff = w->box_backoff ? std::min(2 * w->box_backoff, 64) : 1;
                w->box_skip = w->box_backoff;
                opt = false;
            }
            if (partners)
                if (int rc3 = grow_partners(w)) return rc3;
            if (overflow) {
                // the scene outgrew the layout it was fitted for: refit to
                // the chunk-start positions; if the chunk overflows again,
                // a table twice the size (one more period bit), and once the
                // table is at its limit, shorter chunks
                if (refitted) {
                    bool grown = false;
                    if (int rc3 = grow_table(w, grown)) return rc3;
                    if (!grown) K = K > 1 ? K / 2 : 1;
                }
                if (int rc3 = refit_from_device(w)) return rc3;
                w->refits += 1;
                refitted = true;
            }
            // table headers only rise (atomicMax on generation): the
            // replay's generations must lie above every one the rolled-
            // back chunk used
            w->gen_off += (uint32_t)K + 1u;
            if (int rc3 = gen_guard(w, left + K)) return rc3;
            if (int rc3 = prime(w, dt, e, mu)) return rc3;
        }
        w->c += K;
        left -= K;
    }
    return RB_OK;
}

// A few host threads for the boundary's copies and compares: rb_set_state
// and rb_get_state move 13 doubles per body (6.8 MB at 65,536 bodies), which
// one core copies in ~0.6 ms.  Workers wait on a condition variable; a job
// is cut into pieces taken from an atomic counter by the workers and the
// caller.  Small jobs run inline.
class HostPool {
    std::vector<std::thread> th_;
    std::mutex m_, job_m_;
    std::condition_variable cv_, done_cv_;
    uint64_t gen_ = 0;
    int busy_ = 0;
    bool stop_ = false;
    const std::function<void(size_t, size_t)> *fn_ = nullptr;
    size_t n_ = 0, pieces_ = 0;
    std::atomic<size_t> next_{0}, done_{0};
    void work() {
        for (size_t k; (k = next_.fetch_add(1)) < pieces_;) {
            (*fn_)(n_ * k / pieces_, n_ * (k + 1) / pieces_);
            done_.fetch_add(1);
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> lk(m_);
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            ++busy_;
            lk.unlock();
            work();
            lk.lock();
            --busy_;
            lk.unlock();
            done_cv_.notify_all();
        }
    }

  public:
    HostPool() {
        int want = 8;
        if (const char *ev = getenv("OMP_NUM_THREADS")) want = atoi(ev);
        if (const char *ev = getenv("RBHIP_HOST_THREADS")) want = atoi(ev);
        want = std::max(1, std::min(want, 16));
        for (int k = 1; k < want; ++k) th_.emplace_back([this] { loop(); });
    }
    ~HostPool() {
        { std::lock_guard<std::mutex> lk(m_); stop_ = true; }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    static HostPool &get() { static HostPool p; return p; }
    // fn(lo, hi) over [0, n)
    void run(size_t n, const std::function<void(size_t, size_t)> &fn) {
        if (th_.empty() || n < (size_t(1) << 15)) { fn(0, n); return; }
        std::lock_guard<std::mutex> jl(job_m_);
        {
            std::unique_lock<std::mutex> lk(m_);
            done_cv_.wait(lk, [&] { return busy_ == 0; });     // (no worker still in the last job)
            fn_ = &fn; n_ = n; pieces_ = 4 * (th_.size() + 1);
            next_ = 0; done_ = 0;
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> lk(m_);
        done_cv_.wait(lk, [&] { return done_.load() == pieces_ && busy_ == 0; });
    }
};
// fn(array, lo, hi) over [0, n0) of array 0 and [0, n1) of array 1, in one
// pool run (one wake-up of the workers for both of a state's arrays)
template <typename F> void par_two(size_t n0, size_t n1, const F &fn) {
    HostPool::get().run(n0 + n1, [&](size_t lo, size_t hi) {
        if (lo < n0) fn(0, lo, std::min(hi, n0));
        if (hi > n0) fn(1, std::max(lo, n0) - n0, hi - n0);
    });
}
// dst_k[0, n_k) = src_k[0, n_k), k = 0, 1
void par_copy2(double *d0, const double *s0, size_t n0, double *d1, const double *s1, size_t n1) {
    par_two(n0, n1, [&](int k, size_t lo, size_t hi) {
        if (k == 0) memcpy(d0 + lo, s0 + lo, sizeof(double) * (hi - lo));
        else memcpy(d1 + lo, s1 + lo, sizeof(double) * (hi - lo));
    });
}
bool par_equal2(const double *a0, const double *b0, size_t n0, const double *a1, const double *b1, size_t n1) {
    std::atomic<int> diff{0};
    par_two(n0, n1, [&](int k, size_t lo, size_t hi) {
        const double *a = k ? a1 : a0, *b = k ? b1 : b0;
        if (!diff.load(std::memory_order_relaxed) && memcmp(a + lo, b + lo, sizeof(double) * (hi - lo)) != 0) diff = 1;
    });
    return diff.load() == 0;
}

int io_alloc(rb_world *w) {
    if (w->io_q_h) return RB_OK;
    const size_t nq = (size_t)7 * w->N, nv = (size_t)6 * w->N;
    // mapped and coherent: rb_get_state's kernel stores into them across
    // PCIe, visible to the host once the stream is synchronised
    HIPCHK(hipHostMalloc((void **)&w->io_q_h, sizeof(double) * nq, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostMalloc((void **)&w->io_v_h, sizeof(double) * nv, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer((void **)&w->io_q_hd, w->io_q_h, 0));
    HIPCHK(hipHostGetDevicePointer((void **)&w->io_v_hd, w->io_v_h, 0));
    HIPCHK(hipMalloc((void **)&w->io_q_d, sizeof(double) * nq));
    HIPCHK(hipMalloc((void **)&w->io_v_d, sizeof(double) * nv));
    return RB_OK;
}

template <typename T> StateIO<T> make_io(rb_world *w) {
    StateIO<T> p{};
    p.qpos = w->io_q_d;
    p.qvel = w->io_v_d;
    p.snap = dp<Snap<T>>(w->snap[w->sp()], 0);
    p.quat = w->boxes ? dp<T>(w->qsnap[w->sp()], 0) : nullptr;
    p.st = BodyState<T>{dp<T>(w->state, 0), w->S};
    p.bound = dp<T>(w->consts, 7 * w->Npad);
    p.N = w->N;
    p.lo = w->lo;
    p.n_local = w->n_local;
    p.balls = w->law == RB_LAW_BALLS;
    return p;
}

double bound_of(const rb_scene_desc *d, int64_t b) {
    const double *s = d->size + 3 * b;
    return d->kind[b] == RB_BODY_SPHERE ? s[0] : sqrt(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
}

template <typename T>
int upload_consts(rb_world *w, const rb_scene_desc *d, std::vector<double> &bound) {
    std::vector<T> c((size_t)8 * w->Npad, T(0));
    double rmax = 0;
    bound.assign((size_t)w->N, 0.0);
    for (int64_t b = 0; b < w->N; ++b) {
        const double *s = d->size + 3 * b;
        bound[(size_t)b] = bound_of(d, b);
        if (bound[(size_t)b] > rmax) rmax = bound[(size_t)b];
        c[(size_t)(0 * w->Npad + b)] = (T)d->mass[b];
        for (int k = 0; k < 3; ++k) {
            c[(size_t)((1 + k) * w->Npad + b)] = (T)d->inertia[3 * b + k];
            c[(size_t)((4 + k) * w->Npad + b)] = (T)s[k];
        }
        c[(size_t)(7 * w->Npad + b)] = (T)bound[(size_t)b];
    }
    // cell = 2 x the largest contact reach (2 x 2 rmax): the 2x2x2 query
    w->rmax = rmax;
    const double cs = rmax > 0 ? 4.0 * rmax * 1.001 : 1.0;
    w->inv_cs = 1.0 / cs;
    for (int64_t b = 0; b < w->N; ++b) w->all_spheres = w->all_spheres && d->kind[b] == RB_BODY_SPHERE;
    WCHK(wput(w, w->consts, c.data(), sizeof(T) * c.size()));
    // the tile form's constant types: the distinct (m, I) of the bodies, as
    // the arithmetic type holds them (a record carries its type, so the tile
    // kernel reads m and I from a table in LDS instead of by body id)
    {
        std::vector<std::array<T, 4>> types;
        std::vector<uint8_t> type_of((size_t)w->N, 0);
        for (int64_t b = 0; b < w->N && types.size() <= (size_t)TILE_TYPES; ++b) {
            const std::array<T, 4> t = {(T)d->mass[b], (T)d->inertia[3 * b], (T)d->inertia[3 * b + 1], (T)d->inertia[3 * b + 2]};
            size_t k = 0;
            while (k < types.size() && memcmp(types[k].data(), t.data(), sizeof(t)) != 0) ++k;
            if (k == types.size()) types.push_back(t);
            type_of[(size_t)b] = (uint8_t)k;
        }
        if (types.size() <= (size_t)TILE_TYPES) {
            for (size_t t = 0; t < types.size(); ++t)
                for (int k = 0; k < 4; ++k) w->tile_type_val[t][k] = (double)types[t][k];
            HIPCHK(hipMalloc((void **)&w->tile_type_of, (size_t)w->N));
            WCHK(wput(w, w->tile_type_of, type_of.data(), (size_t)w->N));
            w->tile_ntypes = (int32_t)types.size();
        }
    }
    std::vector<int32_t> k((size_t)w->Npad, 0);
    for (int64_t b = 0; b < w->N; ++b) k[(size_t)b] = d->kind[b];
    WCHK(wput(w, w->kind, k.data(), sizeof(int32_t) * k.size()));
    return RB_OK;
}

void free_world(rb_world *w) {
    if (!w) return;
    (void)hipSetDevice(w->device);
    drop_graphs(w);
    if (w->comm) (void)rccl().CommDestroy(w->comm);
    for (void *q : w->ipc_opened) (void)hipIpcCloseMemHandle(q);
    void *p2pbufs[] = {w->flags, w->epoch, w->peer_snap_dev, w->peer_quat_dev, w->peer_flags_dev, w->bounds, w->push_cnt,
                       w->halo_e};
    for (void *b : p2pbufs)
        if (b) (void)hipFree(b);
    for (auto &pr : w->tev) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
    if (w->opt_save) (void)hipFree(w->opt_save);
    void *tbufs[] = {w->tile_mem, w->tile_fill, w->tile_gen, w->tile_why, w->tile_commits, w->tile_type_of};
    for (void *b : tbufs)
        if (b) (void)hipFree(b);
    if (w->tile_host) (void)hipHostFree(w->tile_host);
    if (w->tile_pub_host) (void)hipHostFree(w->tile_pub_host);
    if (w->defer_host) (void)hipHostFree(w->defer_host);
    if (w->io_q_h) (void)hipHostFree(w->io_q_h);
    if (w->io_v_h) (void)hipHostFree(w->io_v_h);
    if (w->io_q_d) (void)hipFree(w->io_q_d);
    if (w->io_v_d) (void)hipFree(w->io_v_d);
    for (hipEvent_t &e : w->io_ev)
        if (e) (void)hipEventDestroy(e);
    void *bufs[] = {w->snap[0], w->snap[1], w->qsnap[0], w->qsnap[1], w->defer_q, w->defer_cnt, w->state, w->consts, w->kind, w->xfrc, w->gen,
                    w->ids[0], w->ids[1], w->spill[0], w->spill[1], w->pos[0], w->pos[1], w->plist, w->plist_cnt, w->vel[0], w->vel[1], w->err, w->rec_count, w->rec_partner, w->rec_kind,
                    w->rec_dist};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    if (w->err_host) (void)hipHostFree(w->err_host);
    if (w->own_stream) (void)hipStreamDestroy(w->own_stream);
    if (w->cap_stream) (void)hipStreamDestroy(w->cap_stream);
    delete w;
}

}  // namespace

extern "C" {

const char *rb_last_error(void) { return g_err.c_str(); }
const char *rb_version(void) { return "librbhip 0.3 (gfx950, HIP)"; }

int rb_world_create(rb_world **out, const rb_scene_desc *d) {
    ApiScope api_scope_(d ? d->device : -1);
    if (!out || !d) return fail(RB_EINVAL, "null argument");
    *out = nullptr;
    if (d->n_bodies <= 0 || d->n_bodies > (int64_t)INT32_MAX / 2) return fail(RB_EINVAL, "n_bodies out of range");
    if (d->n_planes < 0 || d->n_planes > RB_MAX_PLANES) return fail(RB_EINVAL, "n_planes must be in [0, %d]", RB_MAX_PLANES);
    if (d->dtype != RB_F64 && d->dtype != RB_F32) return fail(RB_EINVAL, "dtype must be RB_F64 or RB_F32");
    if (d->world_size < 1 || d->rank < 0 || d->rank >= d->world_size) return fail(RB_EINVAL, "bad rank/world_size");
    if (!d->kind || !d->mass || !d->inertia || !d->size || (d->n_planes && !d->planes))
        return fail(RB_EINVAL, "null scene array");
    if (d->normal_convention != RB_NORMAL_ORIENTED && d->normal_convention != RB_NORMAL_RAW)
        return fail(RB_EINVAL, "bad normal_convention");
    const int maxp = d->max_partners > 0 ? d->max_partners : 16;
    if (maxp > 32) return fail(RB_EINVAL, "max_partners must be <= 32");
    if (d->bucket_capacity < 0 || d->bucket_capacity > BUCKET_SLOTS)
        return fail(RB_EINVAL, "bucket_capacity must be <= %d", BUCKET_SLOTS);
    for (int64_t b = 0; b < d->n_bodies; ++b) {
        if (d->kind[b] != RB_BODY_SPHERE && d->kind[b] != RB_BODY_BOX) return fail(RB_EINVAL, "body %lld: bad kind", (long long)b);
        if (!(d->mass[b] > 0)) return fail(RB_EINVAL, "body %lld: mass must be > 0", (long long)b);
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RB_ENODEV, "no HIP device available");
    if (d->device < 0 || d->device >= ndev) return fail(RB_ENODEV, "device %d out of range (have %d)", d->device, ndev);

    rb_world *w = new rb_world();
    w->dtype = d->dtype;
    w->esz = d->dtype == RB_F64 ? 8 : 4;
    w->device = d->device;
    w->N = d->n_bodies;
    w->P = d->world_size;
    w->rank = d->rank;
    w->S = (w->N + w->P - 1) / w->P;
    w->Npad = w->S * w->P;
    w->lo = w->S * w->rank;
    const int64_t hi = w->lo + w->S < w->N ? w->lo + w->S : w->N;
    w->n_local = (int32_t)(hi > w->lo ? hi - w->lo : 0);
    w->n_planes = d->n_planes;
    for (int k = 0; k < d->n_planes; ++k)
        for (int j = 0; j < 6; ++j) w->planes[k][j] = d->planes[6 * k + j];
    for (int j = 0; j < 3; ++j) w->g[j] = d->gravity[j];
    w->oriented = d->normal_convention == RB_NORMAL_ORIENTED;
    w->maxp = maxp;
    bool any_box = false;
    for (int64_t b = 0; b < d->n_bodies && !any_box; ++b) any_box = d->kind[b] != RB_BODY_SPHERE;
    // box-capable kernels (sharded worlds exchange the boxes' orientations)
    w->boxes = any_box;
    // records per body: 4 per plane, 1 per sphere partner, up to 4 per
    // partner in scenes with boxes (oracle/rb_oracle_impl.h contact_stride)
    w->maxrec = 4 * w->n_planes + (any_box ? 4 : 1) * w->maxp;
    // worlds with boxes: the cooperative form only up to 4,608 owned bodies
    // (cubes on the incline, per step, helper / plain cooperative / wide:
    // 4,096 8.6 / 10.7 / 11.7 us, 5,184 10.4 / 12.4 / 10.2, 9,216 12.9 /
    // 15.7 / 10.2, 16,384 14.7 (plain) / 12.2; scripts/form_ab.py)
    if (any_box) w->coop_max = 4608;
    if (const char *ev = getenv("RBHIP_COOP_MAX_BODIES")) w->coop_max = atoll(ev);
    if (const char *ev = getenv("RBHIP_WIDE_MAX_BODIES")) w->wide_max = atoll(ev);
    if (const char *ev = getenv("RBHIP_HELP_MAX_BODIES")) w->help_max = atoll(ev);
    if (const char *ev = getenv("RBHIP_WIDE_HELP")) w->wide_help = atoi(ev) != 0;
    // the cell-ordered tile form (rb_tiles.hip): RBHIP_TILE = 0 off, 1 every
    // eligible world, -1 auto, the default (eligible worlds of >=
    // RBHIP_TILE_MIN_BODIES bodies, until their first roll-back): it measures
    // slower than the hashed forms up to 65,536 flat spheres (C3) and faster
    // from 73,984 up
    if (const char *ev = getenv("RBHIP_TILE")) w->tile_mode = atoi(ev) < 0 ? -1 : atoi(ev) ? 1 : 0;
    w->tile_mode_init = w->tile_mode;
    if (const char *ev = getenv("RBHIP_TILE_MIN_BODIES")) w->tile_min_bodies = atoll(ev);
    if (const char *ev = getenv("RBHIP_BOX_OPTIMISTIC")) w->box_opt = atoi(ev) != 0;
    if (const char *ev = getenv("RBHIP_DIAG_OVERFLOW")) w->diag_overflow = atoi(ev);
    // buckets: cooperative worlds (a hash per cell; they also keep a slot
    // snapshot line per bucket) 16 per body; the one-lane and wide forms
    // (linear cell groups, below) 32 per body, so the groups' period spans
    // the scene (C3: 2^21 buckets, 205 m x 102 m x 12.8 m; as fast as 2^23,
    // 16 per body 20 % slower: the period then folds the scene onto itself).
    // At most 2^26 buckets (8 GB of lines per table).
    const bool coop_world = w->n_local <= w->coop_max;
    int64_t want = coop_world ? 16 * w->N : 32 * w->N;
    if (const char *ev = getenv("RBHIP_HASH_FACTOR"))
        if (atoll(ev) > 0) want = atoll(ev) * w->N;
    if (want < 4096) want = 4096;
    // memory cap over both tables (lines, plus slot snapshots in cooperative
    // worlds): RBHIP_HASH_MAX_BYTES, default 8 GiB (1M bodies keep 32 buckets
    // per body, 4M bodies get 8)
    const int64_t per_bucket = 2 * (int64_t)(sizeof(uint32_t) * LINE_WORDS + (coop_world ? w->esz * 4 * LINE_WORDS : 0));
    int64_t cap_bytes = int64_t(8) << 30;
    if (const char *ev = getenv("RBHIP_HASH_MAX_BYTES"))
        if (atoll(ev) > 0) cap_bytes = atoll(ev);
    int64_t hmax = 4096;
    while (hmax * 2 * per_bucket <= cap_bytes && hmax < (int64_t(1) << 26)) hmax *= 2;
    w->H = next_pow2(want) < hmax ? next_pow2(want) : hmax;
    w->hmax = hmax;
    // The one-lane and wide forms group cells 8x8x4, the buckets of a group
    // contiguous (32 KB of lines), and lay the groups out linearly, periodic
    // in 2^lx x 2^ly x 2^lz groups (below): against a hash per cell measured
    // 6 % faster at 65k bodies (flat), 5 % (incline), 12 % at 1M; hashed
    // groups were bimodal (a group collision doubles the bodies of every
    // bucket in both groups and sends waves through the wide form's extra
    // round trip for buckets of 7+ ids).  Those kernels compute
    // the linear layout directly (rb_grid.hpp LAYOUT_LINEAR), so their worlds
    // always use it.  The cooperative form keeps a hash per cell.
    // RBHIP_HASH_GROUP=bx:by:bz sets the group shape (2^bx x 2^by x 2^bz
    // cells); in cooperative worlds bx:by:bz hashes the groups and
    // bx:by:bz:l lays them out linearly.
    int gshape = coop_world ? 0 : 0x233;
    bool linear = !coop_world;
    if (const char *ev = getenv("RBHIP_HASH_GROUP")) {
        int bx = 0, by = 0, bz = 0;
        char mode = 'h';
        if (sscanf(ev, "%d:%d:%d:%c", &bx, &by, &bz, &mode) >= 3 && bx >= 0 && by >= 0 && bz >= 0 && bx + by + bz <= 12)
            gshape = bx | (by << 4) | (bz << 8);
        if (coop_world) linear = mode == 'l';
    }
    auto gbits = [](int g) { return (g & 15) + ((g >> 4) & 15) + ((g >> 8) & 15); };
    // a table too small for the groups: smaller groups (linear), none (hashed)
    while (gshape && (int64_t(1) << gbits(gshape)) > w->H / 4) {
        if (!linear) { gshape = 0; break; }
        for (int sh = 8; sh >= 0; sh -= 4)
            if ((gshape >> sh) & 15) { gshape -= 1 << sh; break; }
    }
    w->group = gshape;
    if (linear) {
        // the group slots split into a period of 2^lx x 2^ly x 2^lz groups (z: at most 8)
        int lg = 0;
        while ((int64_t(1) << (lg + 1)) <= w->H) ++lg;
        lg -= gbits(gshape);
        const int lz = lg / 3 < 3 ? lg / 3 : 3, lx = (lg - lz + 1) / 2, ly = lg - lz - lx;
        w->group |= (lx << 12) | (ly << 16) | (lz << 20) | (1 << 24);
    }
    // heads per 128-byte line (rb_internal.hpp Table): 4 in wide-form worlds
    // (C3 17.4 -> 16.4 us), 2 in one-lane worlds (1M 0.237 -> 0.225 ms; 4
    // there cost 10 % at 262k), 1 in cooperative worlds (no gain measured).
    // The cooperative and wide kernels assume theirs at compile time;
    // RBHIP_HEADS_PER_LINE = 1, 2 or 4 sets the one-lane worlds'.
    const bool wide_world = !coop_world && w->n_local <= w->wide_max;
    int rl = coop_world ? 0 : wide_world ? 2 : 1;
    if (const char *ev = getenv("RBHIP_HEADS_PER_LINE"))
        if (!coop_world && !wide_world) {
            const int r = atoi(ev);
            if (r == 1 || r == 2 || r == 4) rl = r == 1 ? 0 : r == 2 ? 1 : 2;
        }
    w->group |= rl << 25;
    int64_t nsph = 0;
    for (int64_t b = 0; b < w->N; ++b) nsph += d->kind[b] == RB_BODY_SPHERE;
    // algorithmic bytes per body-step: 13 state reals read + 13
    // written + constants (m, I[3], r | h[3])
    w->bytes_per_body_step = (int64_t)w->esz * (26 + 4) + (int64_t)w->esz * ((nsph * 1 + (w->N - nsph) * 3) / w->N);

    auto bail = [&](int rc) { free_world(w); return rc; };
    if (hipSetDevice(w->device) != hipSuccess) return bail(fail(RB_ENODEV, "hipSetDevice(%d) failed", w->device));
#define ALLOC(ptr, bytes)                                                                        \
    do {                                                                                         \
        if (hipMalloc((void **)&(ptr), (bytes)) != hipSuccess)                                   \
            return bail(fail(RB_ENOMEM, "hipMalloc(%lld) failed", (long long)(bytes)));          \
    } while (0)
    for (int k = 0; k < 2; ++k) ALLOC(w->snap[k], (size_t)w->esz * 4 * w->Npad);
    if (w->boxes) {
        for (int k = 0; k < 2; ++k) ALLOC(w->qsnap[k], (size_t)w->esz * 4 * w->Npad);
        ALLOC(w->defer_q, sizeof(int32_t) * (w->S > 0 ? w->S : 1));
        ALLOC(w->defer_cnt, sizeof(int32_t) * 2);
    }
    ALLOC(w->state, (size_t)w->esz * 13 * w->S);
    ALLOC(w->consts, (size_t)w->esz * 8 * w->Npad);
    ALLOC(w->kind, sizeof(int32_t) * w->Npad);
    ALLOC(w->gen, sizeof(uint32_t) * 2);
    // Opt-in (RBHIP_SPLIT=1): large scenes step in two kernels (search,
    // update) joined by a partner list; bit-exact with the oracle on the
    // device (tests/test_gpu_parity.py ragged-scene test) but no faster
    // (DESIGN §5), so the default is the fused one-kernel step.
    const char *split_env = getenv("RBHIP_SPLIT");
    const bool coop = w->n_local <= w->coop_max;
    const bool split = !coop && !w->boxes && split_env && atoi(split_env) == 1;
    if (split) {
        ALLOC(w->plist, sizeof(int32_t) * (w->maxp <= 16 ? 16 : 32) * w->S);
        ALLOC(w->plist_cnt, sizeof(int32_t) * w->S);
    }
    for (int k = 0; k < 2; ++k) {
        ALLOC(w->ids[k], sizeof(uint32_t) * LINE_WORDS * w->H);
        ALLOC(w->spill[k], sizeof(uint32_t) * SPILL_LINE_WORDS * SPILL_LINES);
        // slot snapshots feed the cooperative search only
        if (needs_slot_snapshots(coop, split)) ALLOC(w->pos[k], (size_t)w->esz * 4 * LINE_WORDS * w->H);
    }
    ALLOC(w->err, sizeof(int32_t));
#undef ALLOC
    if (hipHostMalloc((void **)&w->err_host, sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void **)&w->err_host_d, w->err_host, 0) != hipSuccess)
        return bail(fail(RB_ENOMEM, "hipHostMalloc failed"));
    *w->err_host = 0;
    if (hipStreamCreateWithFlags(&w->own_stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&w->cap_stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(RB_ENODEV, "hipStreamCreate failed"));
    w->stream = w->own_stream;
    {
        const std::pair<void *, size_t> zero[] = {
            {w->snap[0], (size_t)w->esz * 4 * w->Npad}, {w->snap[1], (size_t)w->esz * 4 * w->Npad},
            {w->state, (size_t)w->esz * 13 * w->S},
            // bucket headers of generation 0: every table's generation is >= 2
            {w->ids[0], sizeof(uint32_t) * LINE_WORDS * w->H}, {w->ids[1], sizeof(uint32_t) * LINE_WORDS * w->H},
            {w->spill[0], sizeof(uint32_t) * SPILL_LINE_WORDS * SPILL_LINES},
            {w->spill[1], sizeof(uint32_t) * SPILL_LINE_WORDS * SPILL_LINES},
            {w->gen, sizeof(uint32_t) * 2}, {w->err, sizeof(int32_t)}, {w->defer_cnt, sizeof(int32_t) * 2}};
        for (const auto &z : zero)
            if (z.first && hipMemsetAsync(z.first, 0, z.second, w->stream) != hipSuccess)
                return bail(fail(RB_ENODEV, "hipMemsetAsync failed"));
    }
    std::vector<double> bound;
    int rc = w->dtype == RB_F64 ? upload_consts<double>(w, d, bound) : upload_consts<float>(w, d, bound);
    if (rc) return bail(rc);
    w->bound = std::move(bound);
    *out = w;
    return RB_OK;
}

void rb_world_destroy(rb_world *w) {
    ApiScope api_scope_(w ? w->device : -1);
    if (w) {
        (void)hipSetDevice(w->device);
        (void)hipStreamSynchronize(w->stream);
    }
    free_world(w);
}

int rb_set_stream(rb_world *w, void *s) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w) return fail(RB_EINVAL, "null world");
    HIPCHK(hipSetDevice(w->device));
    // work queued on the old stream (a block run's check included)
    // finishes there before later work is ordered on the new one
    if (int rc = finish_pending(w)) return rc;
    HIPCHK(hipStreamSynchronize(w->stream));
    w->stream = (hipStream_t)s;        // NULL = HIP's null stream
    return RB_OK;
}

// The linear cell layout's period (rb_grid.hpp bucket_linear): how the
// table's group bits split over x, y, z.  A split folds the scene onto
// itself where two groups a search reads (the occupied groups and their
// neighbours) land on one run of buckets with at least one of them occupied:
// those buckets then hold bodies of both, i.e. false candidates.  Every
// split is scored by that count of colliding groups and the least is taken;
// ties go to the split that leaves the fewest axes folded (a sheet folded
// along one axis stays collision-free as it moves; folded along two, only
// while the fold happens to miss it), then to the one whose period covers
// the scene's extent most evenly.
// Splitting by extent alone (one bit at a time to the axis the period covers
// least) folded a sheet-like scene — C4's spheres on the incline, whose
// bounding box is deep in z but whose groups are one layer thick — in x and
// y to cover z: 14.8 -> 18.1 us per step; counting collisions keeps C4's
// layout and still fits 4M flat spheres (1.33 -> 0.87 ms) and 32k on a
// 128 x 256 grid (17.9 -> 13.2 us).  Deterministic in the global positions,
// so every rank of a sharded world picks the same split.
static void fit_period(rb_world *w, const double *qpos, bool force) {
    if (!((w->group >> 24) & 1)) return;                 // hashed layouts have no period
    if (const char *ev = getenv("RBHIP_FIT_PERIOD"))
        if (atoi(ev) == 0) return;                       // diagnostic: keep the creation-time split
    const int gb[3] = {w->group & 15, (w->group >> 4) & 15, (w->group >> 8) & 15};
    const int lg = ((w->group >> 12) & 15) + ((w->group >> 16) & 15) + ((w->group >> 20) & 15);
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    std::vector<int64_t> occ;
    occ.reserve((size_t)w->N);
    for (int64_t b = 0; b < w->N; ++b) {
        int64_t g[3];
        bool ok = true;
        for (int d = 0; d < 3; ++d) {
            const double c = qpos[7 * b + d] * w->inv_cs;
            if (!(c == c && c > -1e9 && c < 1e9)) { ok = false; break; }
            lo[d] = c < lo[d] ? c : lo[d];
            hi[d] = c > hi[d] ? c : hi[d];
            g[d] = (int64_t)floor(c) >> gb[d];
            if (g[d] <= -PERIOD_OFF + 1 || g[d] >= PERIOD_OFF - 1) ok = false;
        }
        if (ok) occ.push_back(period_pack(g[0], g[1], g[2]));
    }
    // the split depends on the occupied groups; a call whose groups span
    // the same box as the last fit's (every frame of a per-frame caller:
    // multi_sphere_bounce.py:42 runs once per frame) keeps that fit instead
    // of re-sorting every split (RBHIP_FIT_PERIOD=2 always refits)
    {
        int64_t gb_lo[3] = {INT64_MAX, INT64_MAX, INT64_MAX}, gb_hi[3] = {INT64_MIN, INT64_MIN, INT64_MIN};
        for (int64_t k : occ)
            for (int d = 0; d < 3; ++d) {
                gb_lo[d] = std::min(gb_lo[d], period_unpack(k, d));
                gb_hi[d] = std::max(gb_hi[d], period_unpack(k, d));
            }
        const int64_t key[7] = {gb_lo[0], gb_lo[1], gb_lo[2], gb_hi[0], gb_hi[1], gb_hi[2], (int64_t)w->group};
        const char *ev = getenv("RBHIP_FIT_PERIOD");
        if (!force && w->fit_valid && memcmp(key, w->fit_key, sizeof key) == 0 && !(ev && atoi(ev) == 2)) return;
        memcpy(w->fit_key, key, sizeof key);
        w->fit_valid = true;
    }
    double need[3];
    for (int d = 0; d < 3; ++d)
        need[d] = hi[d] >= lo[d] ? (floor(hi[d]) - floor(lo[d]) + 2) / double(1 << gb[d]) : 1.0;
    int best[3] = {(w->group >> 12) & 15, (w->group >> 16) & 15, (w->group >> 20) & 15};
    std::vector<PeriodSet> sets;
    sets.emplace_back(std::move(occ));
    best_period_split(sets, need, lg, best);
    const int32_t g = (w->group & ~(0xfff << 12)) | (best[0] << 12) | (best[1] << 16) | (best[2] << 20);
    if (g != w->group) {
        w->group = g;
        drop_graphs(w);                                  // the grid is a captured kernel argument
    }
    w->fit_key[6] = (int64_t)w->group;
}

int rb_set_state(rb_world *w, const double *qpos, const double *qvel) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w || !qpos || !qvel) return fail(RB_EINVAL, "null argument");
    HIPCHK(hipSetDevice(w->device));
    if (int rc = finish_pending(w)) return rc;
    if (int rc = io_alloc(w)) return rc;
    const size_t nq = (size_t)7 * w->N, nv = (size_t)6 * w->N;
    // the state the last rb_get_state handed out, handed back unchanged (a
    // per-frame caller: multi_sphere_bounce.py:42 once per frame): nothing
    // to do (one rank: a shard's rows of other ranks are not mirrored)
    if (w->P == 1 && w->mirror_version == w->state_version && par_equal2(qpos, w->io_q_h, nq, qvel, w->io_v_h, nv)) {
        w->io_stats[0] += 1;
        return RB_OK;
    }
    w->io_stats[1] += 1;
    HIPCHK(hipStreamSynchronize(w->stream));     // (a DMA out of the staging may be in flight)
    par_copy2(w->io_q_h, qpos, nq, w->io_v_h, qvel, nv);
    fit_period(w, qpos);
    HIPCHK(hipMemcpyAsync(w->io_q_d, w->io_q_h, sizeof(double) * nq, hipMemcpyHostToDevice, w->stream));
    HIPCHK(hipMemcpyAsync(w->io_v_d, w->io_v_h, sizeof(double) * nv, hipMemcpyHostToDevice, w->stream));
    const hipError_t e = w->dtype == RB_F64 ? launch_state_in<double>(make_io<double>(w), w->stream)
                                            : launch_state_in<float>(make_io<float>(w), w->stream);
    HIPCHK(e);
    w->primed = false;
    w->tile_valid_sp = -1;
    w->tile_fit_valid = false;                           // (refitted at the next tile run)
    if (w->tile_mode_init == -1 && w->tile_mode == 0) {   // a new state: auto mode may try the form again
        w->tile_mode = -1;
        w->tile_backoff = w->tile_skip = 0;
    }
    w->state_version += 1;
    // uploading the staging's bytes yields exactly this state (one rank)
    w->mirror_version = w->P == 1 ? w->state_version : -1;
    return RB_OK;
}

int rb_get_state(rb_world *w, double *qpos, double *qvel) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w || (!qpos && !qvel)) return fail(RB_EINVAL, "null argument");
    HIPCHK(hipSetDevice(w->device));
    if (int rc = finish_pending(w)) return rc;
    if (int rc = io_alloc(w)) return rc;
    // the owned rows only (a shard leaves the others untouched).  Default
    // (RBHIP_IO_OUT=2): one kernel stores the rows straight into the mapped
    // pinned staging (no DMA), then one pool copy out to the caller.  =0: a
    // kernel transposes into the device twin, one DMA, one pool copy; =1:
    // that DMA in four chunks, each copied out as it lands.  65,536 bodies
    // into the caller's arrays, MI355X: 0.21 / 0.22 / 0.28 ms for 2 / 0 / 1
    // (profiles/r04/frame_cost_16threads.log)
    const char *ev = getenv("RBHIP_IO_OUT");
    const int mode = ev ? atoi(ev) : 2;
    const size_t lo = (size_t)w->lo, n = (size_t)w->n_local;
    const size_t nq = qpos ? 7 * n : 0, nv = qvel ? 6 * n : 0;
    if (mode == 2) {
        StateIO<double> pd = make_io<double>(w);
        StateIO<float> pf = make_io<float>(w);
        pd.qpos = pf.qpos = w->io_q_hd;
        pd.qvel = pf.qvel = w->io_v_hd;
        HIPCHK(w->dtype == RB_F64 ? launch_state_out_flat<double>(pd, qpos, qvel, w->stream)
                                  : launch_state_out_flat<float>(pf, qpos, qvel, w->stream));
        HIPCHK(hipStreamSynchronize(w->stream));
        par_copy2(qpos ? qpos + 7 * lo : nullptr, w->io_q_h + 7 * lo, nq, qvel ? qvel + 6 * lo : nullptr,
                  w->io_v_h + 6 * lo, nv);
    } else {
        HIPCHK(w->dtype == RB_F64 ? launch_state_out<double>(make_io<double>(w), qpos, qvel, w->stream)
                                  : launch_state_out<float>(make_io<float>(w), qpos, qvel, w->stream));
        const int nc = mode == 1 && n >= 16384 ? 4 : 1;
        if (nc > 1 && !w->io_ev[0])
            for (hipEvent_t &e : w->io_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        for (int c = 0; c < nc; ++c) {
            const size_t a = lo + n * c / nc, b = lo + n * (c + 1) / nc;
            if (qpos) HIPCHK(hipMemcpyAsync(w->io_q_h + 7 * a, w->io_q_d + 7 * a, sizeof(double) * 7 * (b - a), hipMemcpyDeviceToHost, w->stream));
            if (qvel) HIPCHK(hipMemcpyAsync(w->io_v_h + 6 * a, w->io_v_d + 6 * a, sizeof(double) * 6 * (b - a), hipMemcpyDeviceToHost, w->stream));
            if (nc > 1) HIPCHK(hipEventRecord(w->io_ev[c], w->stream));
        }
        for (int c = 0; c < nc; ++c) {
            const size_t a = lo + n * c / nc, b = lo + n * (c + 1) / nc;
            if (nc > 1) HIPCHK(hipEventSynchronize(w->io_ev[c]));
            else HIPCHK(hipStreamSynchronize(w->stream));
            par_copy2(qpos ? qpos + 7 * a : nullptr, w->io_q_h + 7 * a, qpos ? 7 * (b - a) : 0,
                      qvel ? qvel + 6 * a : nullptr, w->io_v_h + 6 * a, qvel ? 6 * (b - a) : 0);
        }
    }
    w->mirror_version = (w->P == 1 && qpos && qvel) ? w->state_version : -1;
    return RB_OK;
}

int rb_set_xfrc(rb_world *w, const double *xf) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w) return fail(RB_EINVAL, "null world");
    HIPCHK(hipSetDevice(w->device));
    if (int rc = finish_pending(w)) return rc;
    if (!xf) {
        // (graphs capture whether a step reads applied forces)
        if (w->xfrc) { drop_graphs(w); HIPCHK(hipStreamSynchronize(w->stream)); HIPCHK(hipFree(w->xfrc)); w->xfrc = nullptr; }
        return RB_OK;
    }
    if (!w->xfrc) { drop_graphs(w); HIPCHK(hipMalloc(&w->xfrc, (size_t)w->esz * 6 * w->S)); }
    HIPCHK(hipStreamSynchronize(w->stream));             // (steps in flight read the old forces)
    std::vector<double> h((size_t)6 * w->S, 0.0);
    for (int64_t l = 0; l < w->n_local; ++l)
        for (int d = 0; d < 6; ++d) h[(size_t)(d * w->S + l)] = xf[6 * (w->lo + l) + d];
    if (w->dtype == RB_F64) {
        WCHK(wput(w, w->xfrc, h.data(), sizeof(double) * h.size()));
    } else {
        std::vector<float> f(h.begin(), h.end());
        WCHK(wput(w, w->xfrc, f.data(), sizeof(float) * f.size()));
    }
    return RB_OK;
}

int rb_step_async(rb_world *w, int64_t nsteps, double dt, double e, double mu, double thr) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w) return fail(RB_EINVAL, "null world");
    return enqueue_steps(w, nsteps, dt, e, mu, thr);
}

int rb_sync(rb_world *w) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w) return fail(RB_EINVAL, "null world");
    HIPCHK(hipSetDevice(w->device));
    if (int rc = finish_pending(w)) return rc;
    return read_err(w);
}

int rb_step(rb_world *w, int64_t nsteps, double dt, double e, double mu, double thr) {
    ApiScope api_scope_(w ? w->device : -1);
    if (w) w->sync_call = true;
    int rc = rb_step_async(w, nsteps, dt, e, mu, thr);
    if (w) w->sync_call = false;
    if (rc) return rc;
    if ((rc = finish_pending(w))) return rc;
    return read_err(w);
}

int rb_shard_step(rb_world *w, double dt, double e, double mu, double thr) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w) return fail(RB_EINVAL, "null world");
    if (w->law != RB_LAW_MUJOCO) return fail(RB_EUNSUPPORTED, "sharded stepping supports the default contact law only");
    if (!(dt > 0) || !(e >= 0) || !(mu >= 0) || !(thr >= 0)) return fail(RB_EINVAL, "invalid step parameters");
    HIPCHK(hipSetDevice(w->device));
    if (int rc = gen_guard(w, 1)) return rc;
    if (!w->primed) { int rc = prime(w); if (rc) return rc; }
    w->state_version += 1;
    if (w->timing) return timed_launch(w, dt, e, mu, thr);
    return launch_one(w, w->stream, w->c, dt, e, mu, thr);
}

int rb_shard_exchange_done(rb_world *w) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w) return fail(RB_EINVAL, "null world");
    HIPCHK(hipSetDevice(w->device));
    // insert every body not owned here into the next table (own ones went in
    // from the step kernel), reading the freshly exchanged snapshot
    const int nsp = 1 - w->sp();
    hipError_t e = w->dtype == RB_F64
                       ? launch_insert<double>(make_insert<double>(w, nsp, 0, w->N, w->lo, w->lo + w->n_local), w->stream)
                       : launch_insert<float>(make_insert<float>(w, nsp, 0, w->N, w->lo, w->lo + w->n_local), w->stream);
    HIPCHK(e);
    ++w->c;
    return RB_OK;
}

int rb_gpos_buffer(rb_world *w, void **dev_ptr, int64_t *shard_elems, int32_t *elem_bytes) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w) return fail(RB_EINVAL, "null world");
    if (dev_ptr) *dev_ptr = w->snap[1 - w->sp()];
    if (shard_elems) *shard_elems = 4 * w->S;
    if (elem_bytes) *elem_bytes = w->esz;
    return RB_OK;
}

int rb_gquat_buffer(rb_world *w, void **dev_ptr, int64_t *shard_elems, int32_t *elem_bytes) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w) return fail(RB_EINVAL, "null world");
    if (dev_ptr) *dev_ptr = w->boxes ? w->qsnap[1 - w->sp()] : nullptr;
    if (shard_elems) *shard_elems = w->boxes ? 4 * w->S : 0;
    if (elem_bytes) *elem_bytes = w->esz;
    return RB_OK;
}

int rb_comm_unique_id(void *id, int32_t bytes) {
    ApiScope api_scope_(-1);
    if (!id || bytes < (int32_t)sizeof(ncclUniqueId)) return fail(RB_EINVAL, "id buffer must hold %d bytes", (int)sizeof(ncclUniqueId));
    if (!rccl().ok) return fail(RB_ENODEV, "RCCL (librccl.so) not available");
    ncclUniqueId u;
    const ncclResult_t r = rccl().GetUniqueId(&u);
    if (r != ncclSuccess) return fail(RB_ENODEV, "ncclGetUniqueId: %s", rccl().GetErrorString(r));
    memcpy(id, &u, sizeof(u));
    return RB_OK;
}

int rb_shard_comm_init(rb_world *w, const void *id, int32_t bytes) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w || !id || bytes < (int32_t)sizeof(ncclUniqueId)) return fail(RB_EINVAL, "null world or short id");
    if (w->comm) return fail(RB_EINVAL, "communicator already initialised");
    if (!rccl().ok) return fail(RB_ENODEV, "RCCL (librccl.so) not available");
    HIPCHK(hipSetDevice(w->device));
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclResult_t r = rccl().CommInitRank(&w->comm, (int)w->P, u, (int)w->rank);
    if (r != ncclSuccess) { w->comm = nullptr; return fail(RB_ENODEV, "ncclCommInitRank: %s", rccl().GetErrorString(r)); }
    // first collective outside any graph capture (connection setup); the
    // snapshots are replicated, so the in-place gather leaves them unchanged
    if (int rc = rccl_gather(w, w->sp(), w->stream)) return rc;
    HIPCHK(hipStreamSynchronize(w->stream));
    drop_graphs(w);
    return RB_OK;
}

// IPC handles per rank: both snapshots, the mailbox, (box worlds) both
// orientation snapshots
int p2p_nhandles(const rb_world *w) { return w->boxes ? 5 : 3; }

int rb_p2p_handles(rb_world *w, void *out, int64_t cap, int64_t *len) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w || !len) return fail(RB_EINVAL, "null argument");
    const int nh = p2p_nhandles(w);
    const int64_t need = nh * (int64_t)sizeof(hipIpcMemHandle_t);
    *len = need;
    if (!out) return RB_OK;
    if (cap < need) return fail(RB_EINVAL, "handle buffer needs %lld bytes", (long long)need);
    HIPCHK(hipSetDevice(w->device));
    if (!w->flags) {
        // the mailbox, uncached: peers write it over xGMI while this rank's
        // kernels poll and read it
        const MailLayout lay = MailLayout::make(w->P, w->S, w->esz, w->boxes);
        HIPCHK(hipExtMallocWithFlags((void **)&w->flags, (size_t)lay.bytes, hipDeviceMallocUncached));
        WCHK(wfill(w, w->flags, 0, (size_t)lay.bytes));
        HIPCHK(hipStreamSynchronize(w->stream));     // (the peers map it next)
    }
    hipIpcMemHandle_t h[5];
    HIPCHK(hipIpcGetMemHandle(&h[0], w->snap[0]));
    HIPCHK(hipIpcGetMemHandle(&h[1], w->snap[1]));
    HIPCHK(hipIpcGetMemHandle(&h[2], w->flags));
    if (w->boxes) {
        HIPCHK(hipIpcGetMemHandle(&h[3], w->qsnap[0]));
        HIPCHK(hipIpcGetMemHandle(&h[4], w->qsnap[1]));
    }
    memcpy(out, h, need);
    return RB_OK;
}

// both parities of the own cell bounds empty: the next step kernel folds
// into one, the exchange after it resets the other
int reset_bounds(rb_world *w) {
    if (!w->bounds) HIPCHK(hipMalloc((void **)&w->bounds, sizeof(int32_t) * 2 * BOUND_COPIES * BOUND_STRIDE));
    std::vector<int32_t> b((size_t)2 * BOUND_COPIES * BOUND_STRIDE, 0);
    for (int k = 0; k < 2 * BOUND_COPIES; ++k)
        for (int d = 0; d < 3; ++d) { b[(size_t)k * BOUND_STRIDE + d] = INT32_MAX; b[(size_t)k * BOUND_STRIDE + 3 + d] = INT32_MIN; }
    WCHK(wput(w, w->bounds, b.data(), sizeof(int32_t) * b.size()));
    return RB_OK;
}

int rb_p2p_connect(rb_world *w, const void *all, int64_t len) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w || !all) return fail(RB_EINVAL, "null argument");
    const int nh = p2p_nhandles(w);
    const int64_t blob = nh * (int64_t)sizeof(hipIpcMemHandle_t);
    if (len != blob * w->P) return fail(RB_EINVAL, "expected %lld bytes of handles (P blobs)", (long long)(blob * w->P));
    if (!w->flags) return fail(RB_EINVAL, "rb_p2p_handles first");
    if (w->p2p) return fail(RB_EINVAL, "already connected");
    HIPCHK(hipSetDevice(w->device));
    std::vector<void *> snaps(2 * (size_t)w->P, nullptr), quats(2 * (size_t)w->P, nullptr);
    std::vector<int64_t *> flags((size_t)w->P, nullptr);
    const char *b = static_cast<const char *>(all);
    for (int64_t q = 0; q < w->P; ++q) {
        if (q == w->rank) {
            snaps[(size_t)q] = w->snap[0];
            snaps[(size_t)(w->P + q)] = w->snap[1];
            flags[(size_t)q] = w->flags;
            quats[(size_t)q] = w->qsnap[0];
            quats[(size_t)(w->P + q)] = w->qsnap[1];
            continue;
        }
        hipIpcMemHandle_t h[5];
        memcpy(h, b + blob * q, (size_t)blob);
        void *ptr[5] = {};
        for (int k = 0; k < nh; ++k) {
            if (hipIpcOpenMemHandle(&ptr[k], h[k], hipIpcMemLazyEnablePeerAccess) != hipSuccess)
                return fail(RB_ENODEV, "hipIpcOpenMemHandle(rank %lld, buffer %d) failed", (long long)q, k);
            w->ipc_opened.push_back(ptr[k]);
        }
        snaps[(size_t)q] = ptr[0];
        snaps[(size_t)(w->P + q)] = ptr[1];
        flags[(size_t)q] = static_cast<int64_t *>(ptr[2]);
        quats[(size_t)q] = ptr[3];
        quats[(size_t)(w->P + q)] = ptr[4];
    }
    if (w->boxes) {
        HIPCHK(hipMalloc((void **)&w->peer_quat_dev, sizeof(void *) * quats.size()));
        WCHK(wput(w, w->peer_quat_dev, quats.data(), sizeof(void *) * quats.size()));
    }
    HIPCHK(hipMalloc((void **)&w->peer_snap_dev, sizeof(void *) * snaps.size()));
    HIPCHK(hipMalloc((void **)&w->peer_flags_dev, sizeof(int64_t *) * flags.size()));
    HIPCHK(hipMalloc((void **)&w->epoch, sizeof(int64_t)));
    WCHK(wput(w, w->peer_snap_dev, snaps.data(), sizeof(void *) * snaps.size()));
    WCHK(wput(w, w->peer_flags_dev, flags.data(), sizeof(int64_t *) * flags.size()));
    WCHK(wfill(w, w->epoch, 0, sizeof(int64_t)));
    WCHK(wfill(w, w->flags, 0, sizeof(int64_t) * w->P));
    // the own cell bounds (both modes filter the peers' bodies by them)
    if (int rc = reset_bounds(w)) return rc;
    HIPCHK(hipStreamSynchronize(w->stream));         // (the flags zeroed before any peer's step can flag)
    w->p2p = true;
    drop_graphs(w);
    return RB_OK;
}

int rb_p2p_halo(rb_world *w, int32_t enable) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w) return fail(RB_EINVAL, "null world");
    if (!w->p2p) return fail(RB_EINVAL, "rb_p2p_halo before rb_p2p_connect");
    HIPCHK(hipSetDevice(w->device));
    HIPCHK(hipStreamSynchronize(w->stream));
    if (enable) {
        if (!w->push_cnt) HIPCHK(hipMalloc((void **)&w->push_cnt, sizeof(int32_t) * w->P));
        if (!w->halo_e) HIPCHK(hipMalloc((void **)&w->halo_e, sizeof(int64_t)));
        if (int rc = reset_bounds(w)) return rc;
        WCHK(wfill(w, w->push_cnt, 0, sizeof(int32_t) * w->P));
    }
    if (w->halo != (enable != 0)) drop_graphs(w);
    w->halo = enable != 0;
    return RB_OK;
}

int rb_shard_run(rb_world *w, int64_t nsteps, double dt, double e, double mu, double thr) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w) return fail(RB_EINVAL, "null world");
    return enqueue_steps(w, nsteps, dt, e, mu, thr, true);
}

int rb_record_contacts(rb_world *w, int enable) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w) return fail(RB_EINVAL, "null world");
    HIPCHK(hipSetDevice(w->device));
    if (int rc = finish_pending(w)) return rc;
    if (enable && !w->rec_count) {
        const size_t slots = (size_t)w->maxrec * (w->S > 0 ? w->S : 1);
        HIPCHK(hipMalloc((void **)&w->rec_count, sizeof(int32_t) * w->S));
        HIPCHK(hipMalloc((void **)&w->rec_partner, sizeof(int32_t) * slots));
        HIPCHK(hipMalloc((void **)&w->rec_kind, sizeof(int32_t) * slots));
        HIPCHK(hipMalloc(&w->rec_dist, (size_t)w->esz * slots));
        WCHK(wfill(w, w->rec_count, 0, sizeof(int32_t) * w->S));
    }
    if (w->record != (enable != 0)) drop_graphs(w);
    w->record = enable != 0;
    return RB_OK;
}

int rb_get_contacts(rb_world *w, int32_t *counts, int32_t *partner, int32_t *kind, double *dist, int64_t cap,
                    int64_t *total) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w || !counts) return fail(RB_EINVAL, "null argument");
    if (!w->rec_count) return fail(RB_EINVAL, "contact recording was never enabled");
    HIPCHK(hipSetDevice(w->device));
    if (int rc = finish_pending(w)) return rc;
    const size_t slots = (size_t)w->maxrec * w->S;
    std::vector<int32_t> c((size_t)w->S), pa(slots), ki(slots);
    std::vector<double> di(slots);
    HIPCHK(hipMemcpyAsync(c.data(), w->rec_count, sizeof(int32_t) * w->S, hipMemcpyDeviceToHost, w->stream));
    HIPCHK(hipMemcpyAsync(pa.data(), w->rec_partner, sizeof(int32_t) * slots, hipMemcpyDeviceToHost, w->stream));
    HIPCHK(hipMemcpyAsync(ki.data(), w->rec_kind, sizeof(int32_t) * slots, hipMemcpyDeviceToHost, w->stream));
    if (w->dtype == RB_F64) {
        WCHK(wget(w, di.data(), w->rec_dist, sizeof(double) * slots));
    } else {
        std::vector<float> f(slots);
        WCHK(wget(w, f.data(), w->rec_dist, sizeof(float) * slots));
        for (size_t k = 0; k < slots; ++k) di[k] = f[k];
    }
    int64_t t = 0;
    for (int64_t l = 0; l < w->n_local; ++l) {
        const int32_t n = c[(size_t)l] < w->maxrec ? c[(size_t)l] : w->maxrec;
        counts[l] = c[(size_t)l];
        for (int32_t k = 0; k < n; ++k, ++t) {
            if (t < cap) {
                const size_t o = (size_t)l * w->maxrec + k;
                if (partner) partner[t] = pa[o];
                if (kind) kind[t] = ki[o];
                if (dist) dist[t] = di[o];
            }
        }
    }
    if (total) *total = t;
    if (t > cap) return fail(RB_EOVERFLOW, "contact buffer too small: need %lld", (long long)t);
    return RB_OK;
}

static int kat_common(int32_t device, int32_t dtype, int64_t n, const double *in, double *out, int nin, int nout,
                      int which) {
    if (n < 0 || (n && (!in || !out))) return fail(RB_EINVAL, "bad KAT arguments");
    if (dtype != RB_F64 && dtype != RB_F32) return fail(RB_EINVAL, "bad dtype");
    if (n == 0) return RB_OK;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RB_ENODEV, "no HIP device available");
    HIPCHK(hipSetDevice(device));
    double *din = nullptr, *dout = nullptr;
    HIPCHK(hipMalloc(&din, sizeof(double) * nin * n));
    if (hipMalloc(&dout, sizeof(double) * nout * n) != hipSuccess) { (void)hipFree(din); return fail(RB_ENOMEM, "hipMalloc"); }
    hipError_t e = hipMemcpy(din, in, sizeof(double) * nin * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        if (which == 1) e = dtype == RB_F64 ? launch_kat_inertia<double>(n, din, dout, nullptr) : launch_kat_inertia<float>(n, din, dout, nullptr);
        else if (which == 2) e = dtype == RB_F64 ? launch_kat_apply<double>(n, din, dout, nullptr) : launch_kat_apply<float>(n, din, dout, nullptr);
        else if (which == 3) e = dtype == RB_F64 ? launch_kat_pair_impulse<double>(n, din, dout, nullptr) : launch_kat_pair_impulse<float>(n, din, dout, nullptr);
        else if (which == 4) e = dtype == RB_F64 ? launch_kat_narrow<double>(n, din, dout, nullptr) : launch_kat_narrow<float>(n, din, dout, nullptr);
        else e = dtype == RB_F64 ? launch_kat_impulse<double>(n, din, dout, nullptr) : launch_kat_impulse<float>(n, din, dout, nullptr);
    }
    if (e == hipSuccess) e = hipMemcpy(out, dout, sizeof(double) * nout * n, hipMemcpyDeviceToHost);
    (void)hipFree(din);
    (void)hipFree(dout);
    HIPCHK(e);
    return RB_OK;
}

int rb_kat_impulse(int32_t device, int32_t dtype, int64_t n, const double *in, double *out) {
    ApiScope api_scope_(device);
    return kat_common(device, dtype, n, in, out, 24, 10, 0);
}

int rb_kat_inertia(int32_t device, int32_t dtype, int64_t n, const double *in, double *out) {
    ApiScope api_scope_(device);
    return kat_common(device, dtype, n, in, out, 7, 18, 1);
}

int rb_kat_apply(int32_t device, int32_t dtype, int64_t n, const double *in, double *out) {
    ApiScope api_scope_(device);
    return kat_common(device, dtype, n, in, out, 26, 6, 2);
}

int rb_kat_pair_impulse(int32_t device, int32_t dtype, int64_t n, const double *in, double *out) {
    ApiScope api_scope_(device);
    return kat_common(device, dtype, n, in, out, 27, 3, 3);
}

int rb_kat_narrow(int32_t device, int32_t dtype, int64_t n, const double *in, double *out) {
    ApiScope api_scope_(device);
    return kat_common(device, dtype, n, in, out, 22, 33, 4);
}

int rb_set_contact_law(rb_world *w, int32_t law, double tol) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w) return fail(RB_EINVAL, "null world");
    if (law != RB_LAW_MUJOCO && law != RB_LAW_BALLS) return fail(RB_EINVAL, "unknown contact law %d", law);
    if (!(tol >= 0) || !(tol < 1e6)) return fail(RB_EINVAL, "tol must be finite and >= 0");
    // a law change rebuilds the table from the local snapshot, whose rows of
    // bodies no peer pushed to this rank are stale in halo mode
    if (w->halo) return fail(RB_EUNSUPPORTED, "rb_set_contact_law on a halo-exchanging shard");
    if (law == RB_LAW_BALLS) {
        if (!w->all_spheres) return fail(RB_EUNSUPPORTED, "the two-ball law takes spheres only");
        if (w->P != 1) return fail(RB_EUNSUPPORTED, "the two-ball law steps unsharded worlds only");
        const double ground[6] = {0, 0, 1, 0, 0, 0};
        if (w->n_planes > 1 || (w->n_planes == 1 && memcmp(w->planes[0], ground, sizeof(ground)) != 0))
            return fail(RB_EUNSUPPORTED, "the two-ball law's only plane is the z = 0 ground (ball_collision.py:88-90)");
    }
    HIPCHK(hipSetDevice(w->device));
    if (int rc = finish_pending(w)) return rc;
    HIPCHK(hipStreamSynchronize(w->stream));
    if (law == RB_LAW_BALLS && !w->vel[0]) {
        const size_t bytes = (size_t)w->esz * 8 * w->Npad;
        for (int k = 0; k < 2; ++k) {
            if (hipMalloc(&w->vel[k], bytes) != hipSuccess) return fail(RB_ENOMEM, "hipMalloc(%zu) failed", bytes);
            WCHK(wfill(w, w->vel[k], 0, bytes));
        }
    }
    if (w->law == RB_LAW_BALLS && law == RB_LAW_MUJOCO) {
        // the default law keeps positions in the snapshot: restore them
        // from the true positions before the snapshot is read again
        const size_t esz = (size_t)w->esz;
        std::vector<char> st(esz * 13 * w->S), sn(esz * 4 * w->Npad);
        HIPCHK(hipMemcpyAsync(st.data(), w->state, st.size(), hipMemcpyDeviceToHost, w->stream));
        WCHK(wget(w, sn.data(), w->snap[w->sp()], sn.size()));
        for (int64_t l = 0; l < w->n_local; ++l)
            for (int d = 0; d < 3; ++d)
                memcpy(&sn[esz * (4 * (w->lo + l) + d)], &st[esz * ((10 + d) * w->S + l)], esz);
        WCHK(wput(w, w->snap[w->sp()], sn.data(), sn.size()));
    } else if (w->law == RB_LAW_MUJOCO && law == RB_LAW_BALLS) {
        // the other way: the true positions from the snapshot
        const size_t esz = (size_t)w->esz;
        std::vector<char> st(esz * 13 * w->S), sn(esz * 4 * w->Npad);
        HIPCHK(hipMemcpyAsync(st.data(), w->state, st.size(), hipMemcpyDeviceToHost, w->stream));
        WCHK(wget(w, sn.data(), w->snap[w->sp()], sn.size()));
        for (int64_t l = 0; l < w->n_local; ++l)
            for (int d = 0; d < 3; ++d)
                memcpy(&st[esz * ((10 + d) * w->S + l)], &sn[esz * (4 * (w->lo + l) + d)], esz);
        WCHK(wput(w, w->state, st.data(), st.size()));
    }
    w->law = law;
    w->tol = tol;
    w->state_version += 1;
    w->tile_valid_sp = -1;
    // cell = 2 x the largest reach: 2 x 2 rmax, or 2 x (2 rmax + tol)
    const double reach = law == RB_LAW_BALLS ? 2.0 * w->rmax + tol : 2.0 * w->rmax;
    w->inv_cs = 1.0 / (reach > 0 ? 2.0 * reach * 1.001 : 1.0);
    drop_graphs(w);
    w->primed = false;
    return RB_OK;
}

}  // extern "C"

extern "C" {

int rb_world_stats(rb_world *w, int64_t *out, int32_t n) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w || (n > 0 && !out)) return fail(RB_EINVAL, "null argument");
    HIPCHK(hipSetDevice(w->device));
    if (int rc = finish_pending(w)) return rc;
    const bool tile = tile_eligible(w);
    const int form = tile ? FORM_TILE : step_form(w);
    const int64_t v[RB_STATS_COUNT] = {(int64_t)w->graphs.size(), form, w->box_stats[0], w->box_stats[1], w->refits,
                                       w->table_grows, w->H, (int64_t)w->maxp, w->io_stats[0], w->io_stats[1],
                                       w->tile_stats[0], w->tile_stats[1], w->tile_stats[2], w->tile_stats[3],
                                       (int64_t)w->tile_why_seen, (int64_t)w->tile_ntx * w->tile_nty,
                                       (int64_t)w->tile_tc, tile && w->tile_skip == 0 ? 1 : 0, step_form(w)};
    for (int32_t k = 0; k < n && k < RB_STATS_COUNT; ++k) out[k] = v[k];
    return n < RB_STATS_COUNT ? n : RB_STATS_COUNT;
}

int rb_query(rb_world *w, int64_t *n_owned, int64_t *bytes) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w) return fail(RB_EINVAL, "null world");
    if (n_owned) *n_owned = w->n_local;
    if (bytes) *bytes = w->bytes_per_body_step;
    return RB_OK;
}

int rb_tile_config(rb_world *w, int32_t mode, int32_t kmax, double band, int64_t owned) {
    ApiScope api_scope_(w ? w->device : -1);
    (void)kmax;
    (void)band;
    (void)owned;
    if (!w) return fail(RB_EINVAL, "null world");
    if (mode == -1 || mode == 0) return RB_OK;
    if (mode == 1) return fail(RB_EUNSUPPORTED, "rb_tile_config: the tile blocks were retired (librbhip 0.3)");
    return fail(RB_EINVAL, "rb_tile_config: mode must be -1, 0 or 1");
}

int rb_kernel_timing(rb_world *w, int enable, double *avg_ms, int64_t *launches) {
    ApiScope api_scope_(w ? w->device : -1);
    if (!w) return fail(RB_EINVAL, "null world");
    HIPCHK(hipSetDevice(w->device));
    int rc = collect_timing(w);
    if (rc) return rc;
    if (avg_ms) *avg_ms = w->t_n ? w->t_sum_ms / (double)w->t_n : 0.0;
    if (launches) *launches = w->t_n;
    if (enable && !w->timing) { w->t_sum_ms = 0; w->t_n = 0; }
    w->timing = enable != 0;
    return RB_OK;
}

}  // extern "C"
