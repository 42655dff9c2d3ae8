// rb_internal.hpp — shared between the kernels (rb_kernels.hip) and the
// C-ABI implementation (rb_capi.hip).  Not part of the public interface.
#pragma once

#include <cstddef>

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rb {

// error bits accumulated in the world's device error word
enum : int32_t {
    ERR_BUCKET_OVERFLOW = 1,    // broadphase bucket capacity exceeded
    ERR_PARTNER_OVERFLOW = 2,   // more sphere partners than max_partners
    ERR_UNSUPPORTED = 4,        // box-involved pair in range with no box kernel to take it (never raised
                                // since box worlds, sharded or not, always launch one)
    ERR_DOMAIN = 8,             // non-finite / out-of-range position
    ERR_EXCHANGE = 16,          // peer-to-peer exchange: a peer's step did not arrive in time
    ERR_HALO_MOVE = 32,         // halo exchange: a body moved more than one broadphase cell in one step
};

// Step-start snapshot of one body, indexed by global body id: position and
// bounding radius (== the radius for a sphere).  Two snapshot buffers
// ping-pong: a step reads one and writes the other, so every contact test
// sees step-start positions (Jacobi across bodies, multi_sphere_bounce.py:43-46).
// The buffer is also the replicated position buffer of sharded worlds:
// layout [P][S][4], rank r's bodies are the contiguous slice [r*S, r*S+S).
template <typename T> struct alignas(4 * sizeof(T)) Snap { T x, y, z, r; };

// Broadphase buckets: per-cell hash -> one bucket of 128 bytes holding an
// 8-byte header and 30 body ids (laid out in blocks: below), and (cooperative search) slot for slot the
// bodies' snapshots, so a query reads candidates' positions from the bucket
// it already holds instead of chasing ids into the id-indexed snapshot.
//
// The header is (generation << 32) | count.  Every table (the one a step
// reads, the one it fills for the next step) has a generation number that
// only grows; a header with an older generation is an empty bucket.  So a
// query reads count and first two ids with ONE 16-byte load, and nothing is
// ever cleared: an inserter first raises a stale header to (generation, 0)
// with a 64-bit atomicMax, then claims its slot with a 64-bit atomicAdd (two
// atomics of one thread on one address stay in order).  Two line arrays
// alternate with the snapshots.  The generation of the table a step reads
// sits in device memory (gen[step parity]); the step kernel writes the next
// one, so graph replays need no host input.
//
// Heads per line: the buckets are laid out in blocks of R = 1, 2 or 4
// (Grid::super bits 25-26 = log2 R): a block's first 128-byte line holds
// the heads of its R buckets (header and the first 32/R - 2 ids each), the
// further ids of each follow in the block's other lines.  With R > 1 the
// heads of neighbouring cells share lines (under the linear cell layout,
// x-adjacent cells are adjacent buckets): fewer lines fetched per step.
constexpr int LINE_WORDS = 32;               // uint32 words per bucket (head + further ids)
constexpr int HEAD_WORDS = 2;                // the header's words
constexpr int BUCKET_SLOTS = LINE_WORDS - HEAD_WORDS;
constexpr uint32_t BOX_FLAG = 0x80000000u;   // set on ids of box bodies
template <typename T> struct Table {
    uint32_t *line;            // [H / R][R x LINE_WORDS] bucket blocks: heads, then further ids
    Snap<T> *pos;              // [H][LINE_WORDS] slot snapshots (slot s at s); nullptr: not kept
    uint32_t *gen;             // this table's generation (device word)
    uint32_t *spill;           // ids past a full bucket: SPILL_LINES lines of a header (generation
                               // << 32 | count) and SPILL_PAIRS {bucket, tagged id}, a bucket's line
                               // by hash (rb_grid.hpp spill_insert); nullptr: none (an overflow is an error)
};
// A bucket holds 30 ids; a cell with more (a pile-up: C4's sliding rows
// reach 29 by step 700) spills the rest into its table's spill lines: the
// line of the bucket's hash, or the next ones while it is full.  A search
// reads a bucket's spill line(s) only when its count passed its slots.
constexpr int SPILL_LINE_WORDS = 32;
constexpr int SPILL_PAIRS = (SPILL_LINE_WORDS - 2) / 2;   // 15 per line
constexpr int SPILL_LINES = 4096;                         // 512 KB per table
constexpr int SPILL_PROBES = 64;                          // lines tried from the hashed one (<= 960 ids of a bucket)
constexpr int SPILL_GROUP = 1;                            // lines a scan reads per round trip

constexpr int MAX_PLANES = 8;

// contact kinds of box-involved pairs (include/rbhip.h RB_CK_*)
constexpr int CK_SPHERE_BOX = 17;
constexpr int CK_BOX_BOX0 = 32;              // + face-clip point index (< 4)
constexpr int CK_BOX_EDGE = 40;

// Structure-of-arrays body state of this shard.  Positions live in the
// snapshots, except under the two-ball law, whose snapshots hold the next
// step's post-ground positions: its true positions are px, py, pz.
template <typename T> struct BodyState {
    T *base;                           // 13 rows of S reals: qw qx qy qz vx vy vz wx wy wz px py pz
    int64_t S;
    __host__ __device__ T *row(int k) const { return base + k * S; }
    __host__ __device__ T *qw() const { return row(0); }
    __host__ __device__ T *qx() const { return row(1); }
    __host__ __device__ T *qy() const { return row(2); }
    __host__ __device__ T *qz() const { return row(3); }
    __host__ __device__ T *vx() const { return row(4); }
    __host__ __device__ T *vy() const { return row(5); }
    __host__ __device__ T *vz() const { return row(6); }
    __host__ __device__ T *wx() const { return row(7); }
    __host__ __device__ T *wy() const { return row(8); }
    __host__ __device__ T *wz() const { return row(9); }
    __host__ __device__ T *px() const { return row(10); }
    __host__ __device__ T *py() const { return row(11); }
    __host__ __device__ T *pz() const { return row(12); }
};

// Two-ball law: a ball's post-ground velocity and spin, indexed by global id
// (ping-pong with the snapshots).
template <typename T> struct alignas(8 * sizeof(T)) Vel { T vx, vy, vz, wx, wy, wz, pad0, pad1; };

// Per-body constants, global body index (replicated on every rank).
template <typename T> struct BodyConsts {
    const T *base;                     // 8 rows of Npad reals: mass ix iy iz sx sy sz bound
    int64_t Npad;
    const int32_t *kind;
    __host__ __device__ const T *row(int k) const { return base + k * Npad; }
    __host__ __device__ const T *mass() const { return row(0); }
    __host__ __device__ const T *ix() const { return row(1); }      // principal inertia (body frame)
    __host__ __device__ const T *iy() const { return row(2); }
    __host__ __device__ const T *iz() const { return row(3); }
    __host__ __device__ const T *sx() const { return row(4); }      // sphere radius / box half extents
    __host__ __device__ const T *sy() const { return row(5); }
    __host__ __device__ const T *sz() const { return row(6); }
    __host__ __device__ const T *bound() const { return row(7); }   // bounding-sphere radius
};

template <typename T> struct Grid {
    T inv_cs;                          // 1 / cell size
    uint32_t hmask;                    // H - 1 (H power of two)
    int32_t H;
    int32_t super;                     // buckets grouped by super-cell, shape in nibbles (rb_grid.hpp bucket_of);
                                       // bits 25-26: log2 of the heads per line (Table)
};

// Halo exchange (rb_p2p.hip, rb_halo.hpp), for large shards: instead of
// reading every peer's whole slice, each rank PUSHES to each peer only its
// bodies that may come within reach of that peer's bodies — a superset of
// every body the peer's 2x2x2 searches can reach.
//
// The own bounds are accumulated by the step kernel with atomic min/max into
// BOUND_COPIES spread copies (block b uses copy b % BOUND_COPIES, so the
// atomics do not contend on one line), reduced and published by the insert
// kernel (or, before a run's first step, the prime kernel).
constexpr int BOUND_COPIES = 64;
constexpr int BOUND_STRIDE = 32;       // int32 per copy (128 B): min x y z, max x y z, unused
//
// Each rank's mailbox is one uncached allocation, written by the peers over
// xGMI (IPC mappings) and polled / read by this rank:
//   int64  flags[P]             full-read exchange: "step e done" from peer q
//   int64  box[P][6]            halo: peer q's cell bounds, ((e + 1) << 32) | uint32(v)
//   int64  cnt[2][P]            halo: bodies peer q pushed, (e << 32) | count, by step parity
//   uint32 in_ids[2][P][S]      halo: pushed ids by step parity, region q written by peer q
//   Snap   in_snap[2][P][S]     halo: their snapshots
//   T      in_quat[2][P][S][4]  halo, box worlds: the orientations of pushed boxes
// Packing the epoch into every word lets a reader tell a fresh word from a
// stale one without a separate flag (and a release fence before it).
struct MailLayout {
    int64_t o_flags, o_box, o_cnt, bytes;
    int64_t o_ids[2], o_snap[2], o_quat[2];   // o_quat: -1 without boxes
    __host__ __device__ static MailLayout make(int64_t P, int64_t S, int64_t esz, bool boxes) {
        MailLayout m;
        m.o_flags = 0;
        m.o_box = 8 * P;
        m.o_cnt = m.o_box + 48 * P;
        int64_t o = m.o_cnt + 16 * P;
        for (int k = 0; k < 2; ++k) { m.o_ids[k] = o; o += 4 * P * S; }
        o = (o + 255) / 256 * 256;
        for (int k = 0; k < 2; ++k) { m.o_snap[k] = o; o += 4 * esz * P * S; }
        for (int k = 0; k < 2; ++k) {
            m.o_quat[k] = boxes ? o : -1;
            if (boxes) o += 4 * esz * P * S;
        }
        m.bytes = o;
        return m;
    }
};

// The halo push from the step kernels (rb_halo.hpp halo_push): after its
// bodies stepped, a wave appends each one whose new cell lies within two
// cells of a peer's bounds of the step before (published by the peer's
// insert kernel; a peer body moves at most one cell per step, else
// ERR_HALO_MOVE) to that peer's inbox of the step's parity.  mail ==
// nullptr: no push (every other transport).
struct HaloPush {
    char *const *peer_mail;            // [P] each peer's mailbox (own entry unused)
    const char *mail;                  // this rank's mailbox (the peers' bounds)
    int32_t *push_cnt;                 // [P] bodies pushed to each peer this step
    const int64_t *halo_e;             // the epoch of the bounds this step tests against (insert / prime kernel)
    MailLayout lay;
    int64_t S;
    int64_t timeout_ticks;             // s_memrealtime ticks (100 MHz) before ERR_EXCHANGE
    int32_t rank, P;
};

template <typename T> struct StepParams {
    // the first 64 bytes hold everything the step's first loads need, so the
    // prologue fetches them with one scalar load
    const Snap<T> *snap_cur;           // step-start snapshot (read)
    BodyState<T> st;
    BodyConsts<T> cs;
    int32_t n_local, lo;
    int64_t n_global;
    const T *xfrc;                     // [6][S] or nullptr
    int32_t S;
    int32_t n_planes;
    T pn[MAX_PLANES][3], pp[MAX_PLANES][3];
    T g[3];
    T dt, e, mu, thr;
    int32_t oriented;
    Grid<T> grid;
    Snap<T> *snap_next;                // next step's snapshot (own rows written)
    Table<T> cur;                      // broadphase of snap_cur
    Table<T> next;                     // broadphase of snap_next (own ids inserted); line == nullptr: skip
    int32_t *err;
    int64_t *epoch;                    // peer-to-peer exchange: step count, advanced by block 0 (else nullptr)
    int32_t *bounds;                   // halo exchange: [BOUND_COPIES][BOUND_STRIDE] cell bounds of the
                                       // own bodies' new positions (atomic min/max; else nullptr)
    // split form only: sorted partner ids [MAXP][S] and counts [S]
    int32_t *plist, *plist_cnt;
    // two-ball law only (rb_balls.hip)
    const Vel<T> *vel_cur;             // post-ground velocity / spin of snap_cur
    Vel<T> *vel_next;
    T tol;                             // ball_collision.py:102
    int32_t ground;                    // the z = 0 ground plane is present
    // optional contact recording ([n_local][maxrec] slots)
    int32_t *rec_count, *rec_partner, *rec_kind;
    T *rec_dist;
    int32_t maxrec;
    // box-involved pairs (box-capable step kernels only): step-start
    // orientations w x y z by global id, [Npad][4], ping-pong with the
    // snapshots (a partner's state row is updated in place during the step)
    const T *quat_cur;
    T *quat_next;
    // box worlds: the step kernel defers a body with a box-involved partner
    // within bounding range to the box kernel (queue of local indices,
    // counter of this step parity; the box kernel zeroes the other parity's)
    int32_t *defer_q;
    int32_t *defer_cnt;
    int32_t *defer_reset;
    HaloPush halo;                     // fused halo push (halo-exchanging shards)
};

static_assert(offsetof(StepParams<double>, xfrc) == 64 && offsetof(StepParams<float>, xfrc) == 64,
              "prologue fields must fill the first 64 bytes");

template <typename T> struct InsertParams {
    const Snap<T> *snap;               // [Npad]
    const int32_t *kind;               // [Npad]
    int64_t first, count;              // global ids [first, first+count)
    int64_t skip_lo, skip_hi;          // global ids to skip (already inserted)
    Grid<T> grid;
    Table<T> tab;
    int32_t *err;
};

// Peer-to-peer exchange after a sharded step (rb_p2p.hip): every rank reads
// the other ranks' fresh snapshot slices straight from their memory (IPC
// mappings over xGMI), once each peer has flagged its step done, and
// inserts them into its own next table.
template <typename T> struct P2PParams {
    InsertParams<T> ins;               // the local next snapshot's table; skip = own range
    Snap<T> *dst;                      // the local next snapshot (== ins.snap)
    const Snap<T> *const *peer_snap;   // [P] each peer's buffer of this parity (own entry unused)
    int64_t *const *peer_flags;        // [P] each peer's flag array (this rank writes slot rank)
    const int64_t *flags;              // [P] this rank's flags (uncached; peer q writes slot q)
    const int64_t *epoch;              // steps taken (written by the preceding step kernel)
    int32_t rank, P;
    int64_t S;
    int64_t timeout_ticks;             // s_memrealtime ticks (100 MHz) before ERR_EXCHANGE
    // box worlds: each peer's orientation snapshot of this parity ([P], [Npad][4]),
    // copied for the box bodies into the local one (else nullptr)
    const T *const *peer_quat;
    T *qdst;
    // this step's own cell bounds (the step kernel's copies, reduced per
    // block) and the other parity's copies, reset for the next step kernel:
    // a peer's body is inserted only within a cell of them (all of them are
    // still copied into the snapshot)
    const int32_t *bounds;
    int32_t *bounds_reset;
};

// The halo exchange's kernels after the step kernel (insert) and before a
// run's first step (prime)
template <typename T> struct HaloParams {
    InsertParams<T> ins;               // the local next snapshot's table (count, skip unused)
    Snap<T> *dst;                      // the local next snapshot (own rows fresh; pushed rows land here)
    const Snap<T> *own;                // prime: the current snapshot (own rows)
    int32_t *bounds;                   // this step's own-bound copies (from the step kernel)
    int32_t *bounds_reset;             // the other parity's copies: reset for the next step kernel
    int32_t *push_cnt;                 // [P] bodies pushed to each peer this step
    char *const *peer_mail;            // [P] each peer's mailbox (own entry unused)
    const char *mail;                  // this rank's mailbox
    MailLayout lay;
    const int64_t *epoch;
    int64_t *halo_e;                   // written for the next step kernel's pushes
    int32_t rank, P, n_local;
    int64_t lo, S;
    int64_t timeout_ticks;
    // box worlds: the local orientation snapshot of the next step ([Npad][4];
    // own boxes' rows fresh, pushed boxes' rows land here), else nullptr
    T *quat;
};

// ---- the cell-ordered tile form (rb_tiles.hip) -------------------
// Sphere worlds on one rank.  The ground plane (x, y) is cut into columns of
// the hashed forms' cell size (2 x the largest contact reach, so every
// partner of a body lies in the 2 x 2 nearest columns) and the columns into
// square tiles of tc x tc.  Tiles map periodically onto ntx x nty slots;
// one workgroup steps one slot.  Each slot keeps a BIN per step parity: the
// full state of every body the slot stepped, in the column order of the
// slot's tile extended by one ring of columns ((tc + 2)^2 columns, row-major
// from (-1, -1)): a body that left the tile by at most one column lies in
// the ring, i.e. in a neighbouring tile's interior, and that neighbour
// takes it over at the next step.  A step reads the 3 x 3 neighbouring bins
// with coalesced loads, sorts the window of columns (tc + 2)^2 in LDS
// (counts known from the bins' column tables before a record is loaded),
// searches, solves and integrates its own bodies, and writes its next bin
// sorted by column: no atomics on the common path.  A body that moved more
// than a column goes to a small FAR list (one atomic per such body) that
// every slot scans.  Anything the form cannot take (a full bin or window,
// a full far list, too many partners, a bad position) raises ERR_TILE: the
// host rolls the run back and replays it with the hashed-cell forms, which
// also report any real error.
constexpr int32_t ERR_TILE = 1 << 22;
enum : int32_t { TILE_WHY_CAP = 1, TILE_WHY_WINDOW = 2, TILE_WHY_FAR = 4, TILE_WHY_PARTNERS = 8, TILE_WHY_DOMAIN = 16 };
constexpr int TILE_THREADS = 128;        // workgroup size; also the most bodies a slot steps
constexpr int TILE_TC_MIN = 4, TILE_TC_MAX = 8;
constexpr int TILE_OCC3_SLOTS = 1024;    // grids of more slots (> 4 two-wave workgroups per CU) size registers for 3 waves/SIMD
constexpr int TILE_OFFW = 128;           // int32 words per bin's column table (>= (tc + 2)^2 + 1)
constexpr int TILE_WMAX = 384;           // window records a workgroup holds in LDS
constexpr int TILE_FARMAX = 1024;        // far-list capacity
constexpr int TILE_FARWIN = 32;          // far bodies one window holds
constexpr int TILE_STW = 10;             // state reals per record: q (w x y z), v, w
// a record's id word: the body id, and in the top bits its constants' type
// (worlds whose bodies share at most TILE_TYPES distinct (m, I): the kernel
// selects them from its arguments — no memory access between the record's
// arrival and the body's first arithmetic — instead of gathering by id)
constexpr int TILE_ID_BITS = 26;
constexpr int32_t TILE_ID_MASK = (1 << TILE_ID_BITS) - 1;
constexpr int TILE_TYPES = 4;
template <typename T> struct TileBins {
    int32_t *off;                        // [slots][TILE_OFFW] column c at [off[c], off[c + 1]); off[ncol] = count
    Snap<T> *pos;                        // [slots][cap] x y z, bounding radius
    int32_t *id;                         // [slots][cap] id word (id | type << TILE_ID_BITS)
    T *st;                               // [slots][cap][TILE_STW]
    unsigned long long *far_hdr;         // (generation << 32) | count
    Snap<T> *far_pos;                    // [TILE_FARMAX]
    int32_t *far_id;
    T *far_st;                           // [TILE_FARMAX][TILE_STW]
};
template <typename T> struct TileParams {
    TileBins<T> cur, next;
    const uint32_t *gen_cur;             // this step's generation (far-list tags)
    uint32_t *gen_next;                  // written by block 0: gen + 1
    StepParams<T> sp;                    // the physics fields (planes, g, dt, e, mu, thr, oriented, recording,
                                         // err, cs): the same per-body code as the hashed forms (rb_body.hpp)
    T types[TILE_TYPES][4];              // m, ix, iy, iz of each constant type (1..TILE_TYPES)
    int32_t ntypes;
    int32_t tc, ntx, nty, cap;
    T inv_col;                           // 1 / column width
    int32_t *why;                        // TILE_WHY_* bits (diagnostics)
};
// bins <-> the id-ordered state (rb_set_state / rb_get_state / the hashed forms)
template <typename T> struct TileIO {
    TileBins<T> bins;                    // the bins of the current step parity
    const uint32_t *gen;                 // their generation
    Snap<T> *snap;                       // [Npad] the id-ordered snapshot of the same step
    BodyState<T> st;
    const uint8_t *type_of;              // [N] constants' type per body (nullptr: type 0)
    int32_t *fill;                       // [slots][TILE_OFFW] scratch (build)
    int32_t tc, ntx, nty, cap;
    T inv_col;
    int64_t n;
    int32_t *err, *why;
    unsigned long long *commits;         // unbin: runs committed (the host compares)
};
template <typename T> hipError_t launch_tile_step(const TileParams<T> &p, int maxp, hipStream_t s);
template <typename T> hipError_t launch_tile_build(const TileIO<T> &p, hipStream_t s);   // bins zeroed by the caller
template <typename T> hipError_t launch_tile_unbin(const TileIO<T> &p, hipStream_t s);

// launchers (rb_kernels.hip)
// step kernel forms: one lane per body, 8 lanes per body (small scenes), one
// lane per body at one wave per SIMD (mid-size scenes)
enum : int { FORM_ONE = 0, FORM_COOP = 1, FORM_WIDE = 2, FORM_COOP_HELP = 3, FORM_WIDE_HELP = 4, FORM_TILE = 5 };
// boxes: the box-capable instantiation (box-box / sphere-box narrowphase)
template <typename T> hipError_t launch_step(const StepParams<T> &p, int maxp, int form, bool boxes, hipStream_t s);
// the wide form's kernel alone (its own translation unit: scheduled for memory clauses)
template <typename T> hipError_t launch_step_wide(const StepParams<T> &p, int maxp, bool help, hipStream_t s);
template <typename T> hipError_t launch_insert(const InsertParams<T> &p, hipStream_t s);
// rb_set_state / rb_get_state on the device: the reference's AoS rows (qpos
// stride 7: x y z qw qx qy qz; qvel stride 6: v, w; multi_sphere_bounce.py:85-88)
// <-> the SoA state rows and the snapshot (rb_kernels.hip)
template <typename T> struct StateIO {
    double *qpos, *qvel;               // [N][7], [N][6] (device; rows [lo, lo + n_local) for the state)
    Snap<T> *snap;                     // the current snapshot (every body)
    T *quat;                           // box worlds: the current orientation snapshot, else nullptr
    BodyState<T> st;
    const T *bound;                    // [Npad] bounding radii
    int64_t N, lo;
    int32_t n_local;
    int32_t balls;                     // two-ball law: positions are the state's px py pz (the snapshot is post-ground)
};
template <typename T> hipError_t launch_state_in(const StateIO<T> &p, hipStream_t s);
template <typename T> hipError_t launch_state_out(const StateIO<T> &p, bool want_q, bool want_v, hipStream_t s);
template <typename T> hipError_t launch_state_out_flat(const StateIO<T> &p, bool want_q, bool want_v, hipStream_t s);
template <typename T> hipError_t launch_p2p_exchange(const P2PParams<T> &p, hipStream_t s);   // rb_p2p.hip
template <typename T> hipError_t launch_halo_exchange(const HaloParams<T> &p, hipStream_t s); // rb_p2p.hip
template <typename T> hipError_t launch_halo_prime(const HaloParams<T> &p, hipStream_t s);    // rb_p2p.hip
hipError_t launch_publish_err(const int32_t *err, int32_t *host_dev, hipStream_t s,              // rb_p2p.hip
                              const int32_t *why = nullptr, const unsigned long long *commits = nullptr,
                              int64_t *host_tile_dev = nullptr);
template <typename T> hipError_t launch_kat_impulse(int64_t n, const double *in, double *out, hipStream_t s);
template <typename T> hipError_t launch_kat_inertia(int64_t n, const double *in, double *out, hipStream_t s);
template <typename T> hipError_t launch_kat_apply(int64_t n, const double *in, double *out, hipStream_t s);
template <typename T> hipError_t launch_kat_narrow(int64_t n, const double *in, double *out, hipStream_t s);
// two-ball law (rb_balls.hip)
template <typename T> hipError_t launch_ball_step(const StepParams<T> &p, int maxp, hipStream_t s);
template <typename T> hipError_t launch_ball_prime(const StepParams<T> &p, hipStream_t s);
template <typename T> hipError_t launch_kat_pair_impulse(int64_t n, const double *in, double *out, hipStream_t s);

// threads per step-kernel workgroup (the Makefile's WIDE_BLOCK sets it for
// the wide form's unit alone)
#ifndef RB_STEP_BLOCK
#define RB_STEP_BLOCK 64
#endif
constexpr int STEP_BLOCK = RB_STEP_BLOCK;

// lanes per body of the split form's search kernel (1, or 8 = the
// cooperative search, which reads the bucket slot snapshots)
#ifndef RB_SPLIT_G
#define RB_SPLIT_G 1
#endif
constexpr int SPLIT_SEARCH_LANES = RB_SPLIT_G;

// does a world stepping with these forms need bucket slot snapshots?
inline bool needs_slot_snapshots(bool coop, bool split) { return coop || (split && SPLIT_SEARCH_LANES > 1); }

}  // namespace rb
