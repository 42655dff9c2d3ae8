// rb_grid.hpp — the spatial-hash broadphase shared by the step kernels
// (rb_kernels.hip) and the two-ball law (rb_balls.hip): cell and bucket
// maps, slot claims and publication, bucket reads, the 2x2x2 neighbourhood
// and the ascending per-body partner list.  Not part of the public interface.
#pragma once

#include "rb_device.hpp"
#include "rb_internal.hpp"

// write-through (sc1) stores for everything the next step reads: the lines
// leave L2 as they are written, so the end-of-kernel L2 writeback has
// nothing left to flush
#ifndef RB_WT
#define RB_WT 0
#endif
// XCD-aware block order: workgroups are dealt round-robin over the 8 XCDs,
// so block b runs body-block xcd_block(b) and each XCD (own L2) steps one
// contiguous id range = one spatial region of the scene
#ifndef RB_XCD_REMAP
#define RB_XCD_REMAP 0
#endif

// diagnostic builds (rb_kernels.hip lists them): 5 = no candidate snapshot
// loads, 6 = no bucket loads for cells below z = 0
#ifndef RB_ABLATE
#define RB_ABLATE 0
#endif
// per-wave phase stamps (rb_kernels.hip RB_STAMPS builds)
#ifndef STAMP
#define STAMP(k) do {} while (0)
#endif
// candidates whose snapshot loads are issued together
#ifndef RB_QBATCH
#define RB_QBATCH 4
#endif
// cooperative search: bucket slot snapshots loaded with the bucket head,
// before its count is known (most buckets hold one or two bodies)
#ifndef RB_QSPEC
#define RB_QSPEC 2
#endif

namespace rb {

// diagnostic build only (RB_BOUNDS=1): index checks that report and clamp
// instead of faulting
#ifndef RB_BOUNDS
#define RB_BOUNDS 0
#endif
__device__ __forceinline__ int64_t chk(int64_t idx, int64_t n, int line) {
#if RB_BOUNDS
    if (idx < 0 || idx >= n) {
        printf("RB_BOUNDS line %d: index %lld outside [0, %lld) block %d thread %d\n", line, (long long)idx,
               (long long)n, (int)blockIdx.x, (int)threadIdx.x);
        return 0;
    }
#else
    (void)n; (void)line;
#endif
    return idx;
}
#define CHK(idx, n) chk((idx), (n), __LINE__)

// Loads of step-start data (the snapshot, bucket heads and slots, the spill
// list): every writer of it ran in the previous launch, so plain loads.
template <typename V> __device__ __forceinline__ V xld(const V *p) { return *p; }

constexpr uint32_t N_XCD = 8;
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb) {
#if RB_XCD_REMAP
    const uint32_t q = nb / N_XCD, r = nb % N_XCD, x = b % N_XCD;
    return x * q + (x < r ? x : r) + b / N_XCD;
#else
    (void)nb;
    return b;
#endif
}

template <typename V> __device__ __forceinline__ void wt_store(V *ptr, V v) {
#if RB_WT
    __hip_atomic_store(ptr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    *ptr = v;
#endif
}
template <typename T> __device__ __forceinline__ void wt_store(Snap<T> *ptr, const Snap<T> &v) {
    wt_store(&ptr->x, v.x); wt_store(&ptr->y, v.y); wt_store(&ptr->z, v.z); wt_store(&ptr->r, v.r);
}

// cell -> bucket.  Small scenes: one murmur3-finalised hash per cell.
// Large scenes (Grid::super): cells are grouped in aligned 2x2x2
// super-cells — the hash picks the super-cell's run of 8 consecutive buckets
// and the cell's parity bits pick the bucket in it — so a body's 2x2x2
// neighbourhood spans ~3.4 super-cells instead of 8 unrelated buckets and
// its bucket counts share cache lines (measured +10-13% at 1M-4M bodies;
// -3 to -11% below ~300k, where neighbouring inserts then contend on a line).
__device__ __forceinline__ uint32_t bucket_hash(int32_t ix, int32_t iy, int32_t iz) {
    uint32_t h = (uint32_t)ix * 0x8da6b343u + (uint32_t)iy * 0xd8163841u + (uint32_t)iz * 0xcb1ab31fu;
    h ^= h >> 16; h *= 0x85ebca6bu;
    h ^= h >> 13; h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}
// Grid::super packs the group shape: x, y, z bits in nibbles 0, 1, 2 (0x111
// = the 2x2x2 super-cells; 0 = one hash per cell).  Bit 24 set: groups are
// laid out linearly, periodic in 2^lx x 2^ly x 2^lz groups (lx, ly, lz in
// nibbles 3, 4, 5), instead of hashed — no two groups within one period
// share buckets (hashed groups of a compact scene collide with a birthday
// probability near 1, and a collision doubles the bodies of every bucket in
// both groups).
// the linear group layout (Grid::super bit 24)
template <typename T>
__device__ __forceinline__ uint32_t bucket_linear(int32_t ix, int32_t iy, int32_t iz, const Grid<T> &g) {
    const int bx = g.super & 15, by = (g.super >> 4) & 15, bz = (g.super >> 8) & 15, gb = bx + by + bz;
    const int lx = (g.super >> 12) & 15, ly = (g.super >> 16) & 15, lz = (g.super >> 20) & 15;
    const uint32_t sc = ((uint32_t)(ix >> bx) & ((1u << lx) - 1u)) | (((uint32_t)(iy >> by) & ((1u << ly) - 1u)) << lx) |
                        (((uint32_t)(iz >> bz) & ((1u << lz) - 1u)) << (lx + ly));
    const uint32_t in = (uint32_t)(ix & ((1 << bx) - 1)) | ((uint32_t)(iy & ((1 << by) - 1)) << bx) |
                        ((uint32_t)(iz & ((1 << bz) - 1)) << (bx + by));
    return (sc << gb) | in;
}
// Layouts a kernel may assume at compile time: LAYOUT_LINEAR in the one-lane
// and wide forms (their worlds always use it: rb_capi.hip), LAYOUT_ANY
// reads Grid::super
enum : int { LAYOUT_ANY = 0, LAYOUT_LINEAR = 1 };
template <int L = LAYOUT_ANY, typename T>
__device__ __forceinline__ uint32_t bucket_of(int32_t ix, int32_t iy, int32_t iz, const Grid<T> &g) {
    if (L == LAYOUT_LINEAR) return bucket_linear(ix, iy, iz, g);
    if (g.super & 0x1ffffff) {                 // (bits 25-26: heads per line, not the layout)
        const int bx = g.super & 15, by = (g.super >> 4) & 15, bz = (g.super >> 8) & 15, gb = bx + by + bz;
        // arithmetic shifts: floor(c / 2^b)
        const int32_t gx = ix >> bx, gy = iy >> by, gz = iz >> bz;
        uint32_t sc;
        if ((g.super >> 24) & 1) {
            const int lx = (g.super >> 12) & 15, ly = (g.super >> 16) & 15, lz = (g.super >> 20) & 15;
            sc = ((uint32_t)gx & ((1u << lx) - 1u)) | (((uint32_t)gy & ((1u << ly) - 1u)) << lx) |
                 (((uint32_t)gz & ((1u << lz) - 1u)) << (lx + ly));
        } else {
            sc = bucket_hash(gx, gy, gz) & (g.hmask >> gb);
        }
        const uint32_t in = (uint32_t)(ix & ((1 << bx) - 1)) | ((uint32_t)(iy & ((1 << by) - 1)) << bx) |
                            ((uint32_t)(iz & ((1 << bz) - 1)) << (bx + by));
        return (sc << gb) | in;
    }
    return bucket_hash(ix, iy, iz) & g.hmask;
}

// The buckets of a body's 2x2x2 neighbourhood (cells cx + {0, sx}, cy +
// {0, sy}, cz + {0, sz}; bit k of the index picks the neighbour along x, y,
// z).  Under the linear group layout a bucket is a sum of one term per axis,
// so the eight are six terms and eight sums; otherwise bucket_of each.
template <int L = LAYOUT_ANY, typename T>
__device__ __forceinline__ void neighbour_buckets(const Grid<T> &g, int32_t cx, int32_t cy, int32_t cz, int32_t sx,
                                                  int32_t sy, int32_t sz, uint32_t (&b)[8]) {
    if (L == LAYOUT_LINEAR || ((g.super >> 24) & 1)) {
        const int bx = g.super & 15, by = (g.super >> 4) & 15, bz = (g.super >> 8) & 15, gb = bx + by + bz;
        const int lx = (g.super >> 12) & 15, ly = (g.super >> 16) & 15, lz = (g.super >> 20) & 15;
        // term(c) = group bits << (gb + group offset) | in-group bits << in-group offset
        auto term = [](int32_t c, int bc, int lc, int goff, int ioff) {
            return ((((uint32_t)(c >> bc)) & ((1u << lc) - 1u)) << goff) | (((uint32_t)c & ((1u << bc) - 1u)) << ioff);
        };
        const uint32_t x0 = term(cx, bx, lx, gb, 0), x1 = term(cx + sx, bx, lx, gb, 0);
        const uint32_t y0 = term(cy, by, ly, gb + lx, bx), y1 = term(cy + sy, by, ly, gb + lx, bx);
        const uint32_t z0 = term(cz, bz, lz, gb + lx + ly, bx + by), z1 = term(cz + sz, bz, lz, gb + lx + ly, bx + by);
#pragma unroll
        for (int k = 0; k < 8; ++k) b[k] = ((k & 1) ? x1 : x0) | ((k & 2) ? y1 : y0) | ((k & 4) ? z1 : z0);
        return;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
        b[k] = bucket_of(cx + ((k & 1) ? sx : 0), cy + ((k & 2) ? sy : 0), cz + ((k & 4) ? sz : 0), g);
}

// cell coordinates; false for non-finite / out-of-range positions
template <typename T>
__device__ __forceinline__ bool cell_of(T x, T y, T z, T inv_cs, int32_t &ix, int32_t &iy, int32_t &iz) {
    const T fx = x * inv_cs, fy = y * inv_cs, fz = z * inv_cs;
    const T lim = T(1 << 29);
    if (!(absval(fx) < lim && absval(fy) < lim && absval(fz) < lim)) return false;
    ix = (int32_t)__builtin_floor((double)fx);
    iy = (int32_t)__builtin_floor((double)fy);
    iz = (int32_t)__builtin_floor((double)fz);
    return true;
}

// Append a body (tagged id + snapshot) to the bucket of its cell in the
// table of generation gen (rb_internal.hpp Table): an atomicMax raises a
// stale header to (gen, 0), a returning atomicAdd claims the slot
// (claim_slot); the slot is then written (publish_slot).  Split so a caller
// can put independent work between the two and hide the atomic's round trip.
// The Claim keeps the atomic's raw return value and decodes the slot only in
// publish_slot: decoding it in claim_slot, at the join of the caller's
// branches around the claim, made the compiler wait for the atomic right
// there, ahead of all the work placed between the two.
// Bucket b's head (header, then its first ids) and the word of its slot s,
// in blocks of R = 2^rl buckets (rb_internal.hpp Table): the block's first
// line holds the R heads of 32/R words, its other lines the further ids.
__device__ __forceinline__ int grid_rl(int32_t super) { return (super >> 25) & 3; }
__device__ __forceinline__ int64_t head_offset(uint32_t b, int rl) {
    return ((int64_t)(b >> rl) << (5 + rl)) + (int64_t)(b & ((1u << rl) - 1u)) * (LINE_WORDS >> rl);
}
template <typename T> __device__ __forceinline__ uint32_t *head_words(const Table<T> &tab, uint32_t b, int rl) {
    return tab.line + head_offset((uint32_t)CHK(b, RB_BOUNDS ? 1ll << 40 : 0), rl);
}
template <typename T> __device__ __forceinline__ uint32_t *slot_word(const Table<T> &tab, uint32_t b, int s, int rl) {
    if (rl == 0) return tab.line + (int64_t)b * LINE_WORDS + HEAD_WORDS + s;    // one bucket per line
    const int hw = LINE_WORDS >> rl, hid = hw - HEAD_WORDS;         // head words, ids in the head
    const uint32_t r = b & ((1u << rl) - 1u);
    const int64_t blk = (int64_t)(b >> rl) << (5 + rl);
    return tab.line + (s < hid ? blk + (int64_t)r * hw + HEAD_WORDS + s
                               : blk + LINE_WORDS + (int64_t)r * (LINE_WORDS - hw) + (s - hid));
}

struct Claim {
    uint32_t b;
    int32_t ok;                  // 0: not inserted (no table, or a non-finite position)
    unsigned long long old;      // the header before this claim (valid if ok)
    uint32_t gen;
    int32_t rl;                  // the table's log2 heads per line
};
// RL: the table's log2 heads per line when known at compile time (-1: Grid::super)
template <int L = LAYOUT_ANY, int RL = -1, typename T>
__device__ __forceinline__ Claim claim_slot(const Grid<T> &g, const Table<T> &tab, int32_t *err, const Snap<T> &sn,
                                            uint32_t gen) {
    int32_t ix = 0, iy = 0, iz = 0;
    const bool in = cell_of(sn.x, sn.y, sn.z, g.inv_cs, ix, iy, iz);
    if (!in) atomicOr(err, ERR_DOMAIN);
    const uint32_t b = bucket_of<L>(ix, iy, iz, g);
    // no defined value when !in (never decoded then): a constant here would
    // make the join select it against the atomic's return, i.e. wait for it
    unsigned long long old = __builtin_nondeterministic_value(0ull);
    if (in) {
        auto *h = reinterpret_cast<unsigned long long *>(head_words(tab, (uint32_t)CHK(b, g.H), RL >= 0 ? RL : grid_rl(g.super)));
        atomicMax(h, (unsigned long long)gen << 32);
        old = atomicAdd(h, 1ull);
    }
    return {b, in ? 1 : 0, old, gen, RL >= 0 ? RL : grid_rl(g.super)};
}
// An id past a full bucket: (bucket, id) into the table's spill lines — the
// line of the bucket's hash, claimed like a slot (generation-tagged count,
// atomicMax then atomicAdd), or while that line is full the next ones (up to
// SPILL_PROBES).  The counts keep rising past a line's pairs, so a reader
// knows to go on to the next line.
__device__ __forceinline__ uint32_t spill_line_of(uint32_t b) {
    uint32_t h = b * 0x9e3779b1u;
    h ^= h >> 15;
    return h & (uint32_t)(SPILL_LINES - 1);
}
template <typename T>
__device__ __forceinline__ void spill_insert(const Table<T> &tab, int32_t *err, uint32_t b, uint32_t tagged_id,
                                          uint32_t gen) {
    if (!tab.spill) { atomicOr(err, ERR_BUCKET_OVERFLOW); return; }
    uint32_t ln = spill_line_of(b);
#pragma unroll 1
    for (int pr = 0; pr < SPILL_PROBES; ++pr, ln = (ln + 1) & (uint32_t)(SPILL_LINES - 1)) {
        uint32_t *line = tab.spill + (int64_t)ln * SPILL_LINE_WORDS;
        auto *h = reinterpret_cast<unsigned long long *>(line);
        atomicMax(h, (unsigned long long)gen << 32);
        const unsigned long long old = atomicAdd(h, 1ull);
        const uint32_t k = (uint32_t)(old >> 32) == gen ? (uint32_t)old : (uint32_t)SPILL_PAIRS;
        if (k < (uint32_t)SPILL_PAIRS) {
            wt_store(line + 2 + 2 * k, b);
            wt_store(line + 3 + 2 * k, tagged_id);
            return;
        }
    }
    atomicOr(err, ERR_BUCKET_OVERFLOW);
}
// f(tagged id) for each spilled id of bucket b (buckets whose header count
// passed BUCKET_SLOTS only: the rare path): its hashed line and the ones
// after it, SPILL_GROUP lines (one round trip) at a time, until a line read
// had not overflowed
template <typename T, typename F>
__device__ __forceinline__ void spill_scan(const Table<T> &tab, uint32_t gen, uint32_t b, F f) {
    if (!tab.spill) return;
    const uint32_t l0 = spill_line_of(b);
#pragma unroll 1
    for (int pr = 0; pr < SPILL_PROBES; pr += SPILL_GROUP) {
        uint4 v[SPILL_GROUP][SPILL_LINE_WORDS / 4];
#pragma unroll
        for (int g = 0; g < SPILL_GROUP; ++g) {
            const uint32_t ln = (l0 + (uint32_t)(pr + g)) & (uint32_t)(SPILL_LINES - 1);
            const uint4 *l = reinterpret_cast<const uint4 *>(tab.spill + (int64_t)ln * SPILL_LINE_WORDS);
#pragma unroll
            for (int q = 0; q < SPILL_LINE_WORDS / 4; ++q) v[g][q] = xld(l + q);
        }
#pragma unroll
        for (int g = 0; g < SPILL_GROUP; ++g) {
            const uint32_t n = v[g][0].y != gen ? 0u : v[g][0].x;
#pragma unroll
            for (int k = 0; k < SPILL_PAIRS; ++k) {
                // pair k: words 2 + 2k, 3 + 2k of the line
                const uint4 &c = v[g][(2 + 2 * k) / 4];
                const uint32_t wb = ((2 + 2 * k) & 3) == 0 ? c.x : c.z;
                const uint32_t wi = ((2 + 2 * k) & 3) == 0 ? c.y : c.w;
                if ((uint32_t)k < n && wb == b) f(wi);
            }
            if (n <= (uint32_t)SPILL_PAIRS) return;
        }
    }
}
// the header's count passed the slots: bucket b has spilled ids
// (diagnostic builds RB_SPILL=0: searches ignore the spill list)
#ifndef RB_SPILL
#define RB_SPILL 1
#endif
__device__ __forceinline__ bool head_spilled(const uint4 &h, uint32_t gen) {
    return RB_SPILL && h.y == gen && h.x > (uint32_t)BUCKET_SLOTS;
}

template <int RL = -1, typename T>
__device__ __forceinline__ void publish_slot(const Table<T> &tab, int32_t *err, Claim c, const Snap<T> &sn,
                                             uint32_t tagged_id) {
    if (!c.ok) return;
    // after the max the header carries gen (no later generation writes this
    // table before the next step's launch)
    const int32_t slot = (uint32_t)(c.old >> 32) == c.gen ? (int32_t)(uint32_t)c.old : BUCKET_SLOTS;
    if (slot >= BUCKET_SLOTS) {
        if ((uint32_t)(c.old >> 32) == c.gen) spill_insert(tab, err, c.b, tagged_id, c.gen);
        else atomicOr(err, ERR_BUCKET_OVERFLOW);
        return;
    }
    wt_store(slot_word(tab, c.b, slot, RL >= 0 ? RL : c.rl), tagged_id);
    if (tab.pos) wt_store(tab.pos + (int64_t)c.b * LINE_WORDS + slot, sn);
}
template <typename T>
__device__ __forceinline__ void insert_id(const Grid<T> &g, const Table<T> &tab, int32_t *err, const Snap<T> &sn,
                                          uint32_t tagged_id, uint32_t gen) {
    publish_slot(tab, err, claim_slot(g, tab, err, sn, gen), sn, tagged_id);
}

// A bucket's header and first two ids in one 16-byte load; count = 0 unless
// the header carries the table's generation (clamped to the slots).
template <typename T>
__device__ __forceinline__ uint4 bucket_head(const Table<T> &tab, uint32_t b, int rl) {
    return xld(reinterpret_cast<const uint4 *>(head_words(tab, b, rl)));
}
__device__ __forceinline__ int32_t head_count(const uint4 &h, uint32_t gen) {
    return h.y != gen ? 0 : h.x < (uint32_t)BUCKET_SLOTS ? (int32_t)h.x : BUCKET_SLOTS;
}
template <typename T>
__device__ __forceinline__ uint32_t bucket_id(const Table<T> &tab, uint32_t b, const uint4 &h, int s, int rl) {
    return s == 0 ? h.z : s == 1 ? h.w : xld(slot_word(tab, b, s, rl));
}

// The 2x2x2 cell neighbourhood: cell size = 2 x the largest contact reach
// (2 x max bounding diameter), so every partner lies in this body's cell or
// its neighbour on the nearer side along each axis.
template <typename T>
__device__ __forceinline__ bool neighbourhood(const StepParams<T> &p, V3<T> x, int32_t &cx, int32_t &cy, int32_t &cz,
                                              int32_t &sx, int32_t &sy, int32_t &sz) {
    if (!cell_of(x.x, x.y, x.z, p.grid.inv_cs, cx, cy, cz)) return false;
    sx = (x.x * p.grid.inv_cs - (T)cx < T(0.5)) ? -1 : 1;
    sy = (x.y * p.grid.inv_cs - (T)cy < T(0.5)) ? -1 : 1;
    sz = (x.z * p.grid.inv_cs - (T)cz < T(0.5)) ? -1 : 1;
    return true;
}

// Insert partner id j into a per-body list kept ascending in LDS.
template <int MAXP>
__device__ __forceinline__ void list_insert(int32_t *s_id, int stride, int slot, int32_t &np_, int32_t j,
                                            bool &overflow) {
    int pos = np_;
    while (pos > 0) {
        const int32_t prev = s_id[(pos - 1) * stride + slot];
        if (prev == j) return;                       // reached through two hashed cells
        if (prev < j) break;
        --pos;
    }
    if (np_ >= MAXP) { overflow = true; return; }
    for (int t = np_; t > pos; --t) s_id[t * stride + slot] = s_id[(t - 1) * stride + slot];
    s_id[pos * stride + slot] = j;
    ++np_;
}

// One lane per body: the 8 bucket heads (count and first 2 ids) are loaded
// together, then candidates in batches of RB_QBATCH (snapshot
// loads in flight together); hit(tagged id, snapshot) decides a partner.
// The partners go to the body's LDS column of s_id in ascending id order.
// Returns the partner count.
template <typename T, int MAXP, int L = LAYOUT_ANY, typename Hit>
__device__ __forceinline__ int32_t search_buckets(const StepParams<T> &p, int32_t i, V3<T> x, int32_t *s_id,
                                                  int tid, uint32_t gen, Hit hit) {
    constexpr int NB = STEP_BLOCK;
    int32_t cx, cy, cz, sx, sy, sz;
    if (!neighbourhood(p, x, cx, cy, cz, sx, sy, sz)) { atomicOr(p.err, ERR_DOMAIN); return 0; }
    uint32_t b[8];
    int32_t c[8];
    uint4 hd[8];
    neighbour_buckets<L>(p.grid, cx, cy, cz, sx, sy, sz, b);
    const int rl = grid_rl(p.grid.super);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (RB_ABLATE == 6 && (k & 4) && cz + sz < 0) hd[k] = uint4{0u, 0u, 0u, 0u};
        else hd[k] = bucket_head(p.cur, (uint32_t)CHK(b[k], p.grid.H), rl);
    }
    STAMP(8);
    int32_t total = 0;
    uint32_t spm = 0;                                 // buckets with spilled ids
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        int32_t n = head_count(hd[k], gen);
#pragma unroll
        for (int j = 0; j < k; ++j)
            if (b[j] == b[k]) n = 0;                  // two cells hashed to one bucket: visit once
        c[k] = n;
        total += n;
        if (n > 0 && head_spilled(hd[k], gen)) spm |= 1u << k;
    }
    int32_t np_ = 0;
    bool overflow = false;
    // at least one batch, even for total == 0 (its candidates are then this
    // body itself, which hit() rejects): the head loads are used on every
    // path, so the compiler cannot sink them under a total > 0 branch, behind
    // the wait for the counts (one dependent round trip more per body)
    int base = 0;
    do {
        uint32_t tj[RB_QBATCH];
        Snap<T> sn[RB_QBATCH];
#pragma unroll
        for (int u = 0; u < RB_QBATCH; ++u) {
            int32_t rem = base + u;
            uint32_t t = (uint32_t)i;
            const uint32_t *at = nullptr;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (rem >= 0 && rem < c[k]) {
                    if (rem == 0) t = hd[k].z;
                    else if (rem == 1) t = hd[k].w;
                    else at = slot_word(p.cur, b[k], rem, rl);
                }
                rem -= c[k];
            }
            if (base + u < total && at) t = xld(at);
            tj[u] = (base + u < total) ? t : (uint32_t)i;
        }
        // the id-indexed snapshot: ids are spatially coherent, so a wave's
        // candidates share lines (cheaper than bucket slots at this scale).
        // The body itself (always in its own cell's bucket) and the padding
        // of the last batch are no candidates: their lanes load nothing.
#pragma unroll
        for (int u = 0; u < RB_QBATCH; ++u) {
            sn[u] = Snap<T>{RB_ABLATE == 5 ? x.x + T(1000) : x.x, x.y, x.z, T(0)};
            if ((tj[u] & ~BOX_FLAG) != (uint32_t)i && RB_ABLATE != 5)
                sn[u] = xld(p.snap_cur + CHK(tj[u] & ~BOX_FLAG, p.n_global));
        }
#pragma unroll
        for (int u = 0; u < RB_QBATCH; ++u)
            if (hit(tj[u], sn[u]))
                list_insert<MAXP>(s_id, NB, tid, np_, (int32_t)(tj[u] & ~BOX_FLAG), overflow);
        base += RB_QBATCH;
        if (base == RB_QBATCH) STAMP(9);
    } while (base < total);
    if (spm) {                                        // rare: ids past full buckets
#pragma unroll 1
        for (int k = 0; k < 8; ++k) {
            if (!((spm >> k) & 1u)) continue;
            spill_scan(p.cur, gen, b[k], [&](uint32_t t) {
                const uint32_t j = t & ~BOX_FLAG;
                if (j == (uint32_t)i) return;
                if (hit(t, xld(p.snap_cur + CHK(j, p.n_global)))) list_insert<MAXP>(s_id, NB, tid, np_, (int32_t)j, overflow);
            });
        }
    }
    STAMP(10);
    if (overflow) atomicOr(p.err, ERR_PARTNER_OVERFLOW);
    return np_;
}

// Wide form: the first WIDE_HPOS hits' snapshots stay in LDS (s_hpos, in
// discovery order), so the solve does not gather them a second time;
// s_didx maps a sorted list position to its discovery index (>= WIDE_HPOS:
// gathered again).  RB_WIDE_LDSPOS=0: always gathered.
#ifndef RB_WIDE_LDSPOS
#define RB_WIDE_LDSPOS 1
#endif
constexpr int WIDE_HPOS = 8;
// the rare path (buckets of 7+ bodies) software-pipelined over its batches,
// its cursor in registers (2; 1: the cursor walked through LDS, C4 pile-up
// 60.5 -> 55.1 us for 2, C3 unchanged, profiles/r04/rare_cursor_*; 0: each
// batch's ids, then its snapshots)
#ifndef RB_WIDE_PIPE
#define RB_WIDE_PIPE 2
#endif
// diagnostic (0): the wide search skips buckets' ids past the head (wrong
// for a bucket of 7+ bodies); measures the rare path's code footprint
#ifndef RB_WIDE_MORE
#define RB_WIDE_MORE 1
#endif

template <int MAXP, typename T>
__device__ __forceinline__ void list_insert_pos(int32_t *s_id, uint8_t *s_didx, Snap<T> *s_hpos, int stride, int slot,
                                                int32_t &np_, int32_t &nh, int32_t j, const Snap<T> &sn,
                                                bool &overflow) {
    int pos = np_;
    while (pos > 0) {
        const int32_t prev = s_id[(pos - 1) * stride + slot];
        if (prev == j) return;
        if (prev < j) break;
        --pos;
    }
    if (np_ >= MAXP) { overflow = true; return; }
    for (int t = np_; t > pos; --t) {
        s_id[t * stride + slot] = s_id[(t - 1) * stride + slot];
        s_didx[t * stride + slot] = s_didx[(t - 1) * stride + slot];
    }
    s_id[pos * stride + slot] = j;
    s_didx[pos * stride + slot] = (uint8_t)(nh < 255 ? nh : 255);
    if (nh < WIDE_HPOS) s_hpos[nh * stride + slot] = sn;
    ++nh;
    ++np_;
}

// ---- wide one-lane search (one wave per SIMD, rb_kernels.hip step_kernel_wide)
// A bucket head of 32 bytes: header and the first WIDE_HEAD_IDS ids.
constexpr int WIDE_HEAD_IDS = 6;                    // (heads are at least 32 bytes: R <= 4)
#ifndef RB_WIDE_QBATCH
#define RB_WIDE_QBATCH 12
#endif
constexpr int WIDE_QBATCH = RB_WIDE_QBATCH;         // candidates per round trip (8: C3 15.9 us, 32k 12.8; 12: 15.6, 12.3; 16 spills)
constexpr int WIDE_MAXC = 8 * WIDE_HEAD_IDS;        // head candidates listed in LDS
struct Head6 { uint4 a, b; };
template <typename T>
__device__ __forceinline__ Head6 bucket_head6(const Table<T> &tab, uint32_t b, int rl) {
    const uint4 *l = reinterpret_cast<const uint4 *>(head_words(tab, b, rl));
    return Head6{xld(l), xld(l + 1)};
}
template <int S> __device__ __forceinline__ uint32_t head6_id(const Head6 &h) {
    static_assert(S >= 0 && S < WIDE_HEAD_IDS, "head slot");
    return S == 0 ? h.a.z : S == 1 ? h.a.w : S == 2 ? h.b.x : S == 3 ? h.b.y : S == 4 ? h.b.z : h.b.w;
}

// The same contact set and order as search_buckets, with fewer dependent
// round trips: the 8 heads carry 6 ids each, so candidates of the first 6
// slots are known after the head round trip; they are listed (the body
// itself left out) in the lane's LDS column s_cand and their snapshots
// fetched WIDE_QBATCH at a time.  Slots past 6 (rare: a bucket of 7+
// bodies) are read afterwards, ids then snapshots.  overlap() runs under
// the head loads.  Meant for one wave per SIMD: it holds many registers.
// The lane's partner list (its s_id column, np entries, distinct) sorted
// ascending in registers: padded to MAXP with INT32_MAX, a bitonic network
// (MAXP = 16 or 32: 80 / 240 compare-exchanges, no memory round trip), then
// written back; with s_didx, each sorted entry's discovery index among the
// first WIDE_HPOS discovered (255 past them), from those ids kept aside.
constexpr int WIDE_RANK_MAX = 8;                     // longer lists: the bitonic network
template <int MAXP>
__device__ __forceinline__ void sort_partners_bitonic(int32_t *s_id, uint8_t *s_didx, int stride, int slot, int32_t np,
                                                      int32_t nh) {
    static_assert(MAXP == 16 || MAXP == 32, "bitonic: a power of two");
    int32_t a[MAXP];
#pragma unroll
    for (int q = 0; q < MAXP; ++q) a[q] = q < np ? s_id[q * stride + slot] : INT32_MAX;
    int32_t first[WIDE_HPOS];
#pragma unroll
    for (int q = 0; q < WIDE_HPOS; ++q) first[q] = q < nh ? a[q] : -1;
#pragma unroll
    for (int k = 2; k <= MAXP; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
            for (int q = 0; q < MAXP; ++q) {
                const int l = q ^ j;
                if (l > q) {
                    const int32_t lo = min(a[q], a[l]), hi = max(a[q], a[l]);
                    const bool up = (q & k) == 0;
                    a[q] = up ? lo : hi;
                    a[l] = up ? hi : lo;
                }
            }
#pragma unroll
    for (int q = 0; q < MAXP; ++q)
        if (q < np) {
            s_id[q * stride + slot] = a[q];
            if (s_didx) {
                int d = 255;
#pragma unroll
                for (int f = 0; f < WIDE_HPOS; ++f) d = first[f] == a[q] ? f : d;
                s_didx[q * stride + slot] = (uint8_t)d;
            }
        }
}

template <typename T, int MAXP, typename Hit, typename Overlap>
__device__ __forceinline__ int32_t search_buckets_wide(const StepParams<T> &p, int32_t i, V3<T> x, int32_t *s_id,
                                                       uint32_t *s_cand, uint8_t *s_didx, Snap<T> *s_hpos, int tid,
                                                       uint32_t gen, Hit hit, Overlap overlap) {
    constexpr int NB = STEP_BLOCK;
    constexpr int QB = WIDE_QBATCH;
    int32_t cx, cy, cz, sx, sy, sz;
    if (!neighbourhood(p, x, cx, cy, cz, sx, sy, sz)) {
        atomicOr(p.err, ERR_DOMAIN);
        overlap();                                // (on both paths: measured 2-4 % faster at 32k-65k bodies)
        return 0;
    }
    uint32_t b[8];
    int32_t c[8];
    Head6 hd[8];
    neighbour_buckets<LAYOUT_LINEAR>(p.grid, cx, cy, cz, sx, sy, sz, b);
    constexpr int rl = 2;                         // heads per line: wide-form worlds 4 (rb_capi.hip)
#pragma unroll
    for (int k = 0; k < 8; ++k) hd[k] = bucket_head6(p.cur, (uint32_t)CHK(b[k], p.grid.H), rl);
    // the head loads issue here, before the body work: left to itself the
    // scheduler hoisted the work (and its waits for the state loads) above
    // them, and the head round trip started only after it
    __builtin_amdgcn_sched_barrier(0);
    overlap();                                    // body work under the head loads
    STAMP(8);
    int32_t n = 0;
    bool more = false;
    uint32_t spm = 0;                                 // buckets with spilled ids
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        int32_t m = head_count(hd[k].a, gen);
#pragma unroll
        for (int j = 0; j < k; ++j)
            if (b[j] == b[k]) m = 0;                  // two cells hashed to one bucket: visit once
        c[k] = m;
        more |= m > WIDE_HEAD_IDS;
        if (m > 0 && head_spilled(hd[k].a, gen)) spm |= 1u << k;
        // branch-free: every id is written at the list's end, which advances
        // only for a listed one (the last write lands at index <= WIDE_MAXC-1)
#define RB_WIDE_LIST(S)                                                           \
        {                                                                         \
            const uint32_t t = head6_id<S>(hd[k]);                                \
            s_cand[n * NB + tid] = t;                                             \
            n += (S < m && (t & ~BOX_FLAG) != (uint32_t)i) ? 1 : 0;               \
        }
        RB_WIDE_LIST(0) RB_WIDE_LIST(1) RB_WIDE_LIST(2) RB_WIDE_LIST(3) RB_WIDE_LIST(4) RB_WIDE_LIST(5)
#undef RB_WIDE_LIST
    }
    int32_t np_ = 0, nh = 0;
    bool overflow = false;
    // hits are appended in discovery order and ranked by id once the search
    // is done (below): sorting each into place as it came cost a dependent
    // LDS read per list entry passed — C4's pile-ups, up to 28 partners,
    // spent ~40k cycles per step there
    auto append = [&](int32_t j, const Snap<T> &sn) {
        if (np_ >= MAXP) { overflow = true; return; }
        s_id[np_ * NB + tid] = j;
        if (RB_WIDE_LDSPOS) {
            if (nh < WIDE_HPOS) s_hpos[nh * NB + tid] = sn;
            ++nh;
        }
        ++np_;
    };
    // candidates WIDE_QBATCH at a time; the first batch is issued by every
    // lane (padding = the body itself, which loads nothing): measured 2-7 %
    // faster at 32k-65k bodies than a loop all of whose batches are
    // conditional on the lane's candidate count
    auto batch = [&](int base) {
        uint32_t tj[QB];
        Snap<T> sn[QB];
#pragma unroll
        for (int u = 0; u < QB; ++u) tj[u] = base + u < n ? s_cand[(base + u) * NB + tid] : (uint32_t)i;
#pragma unroll
        for (int u = 0; u < QB; ++u) {
            sn[u] = Snap<T>{x.x, x.y, x.z, T(0)};
            if ((tj[u] & ~BOX_FLAG) != (uint32_t)i) sn[u] = xld(p.snap_cur + CHK(tj[u] & ~BOX_FLAG, p.n_global));
        }
#pragma unroll
        for (int u = 0; u < QB; ++u)
            if (base + u < n && hit(tj[u], sn[u])) {
                append((int32_t)(tj[u] & ~BOX_FLAG), sn[u]);
            }
    };
    batch(0);
    for (int base = QB; base < n; base += QB) batch(base);
    STAMP(9);
#if RB_WIDE_PIPE == 2
    if (RB_WIDE_MORE && more) {
        // buckets of 7+ bodies, software-pipelined and batched across
        // buckets as below, with the cursor in registers: the ids past the
        // heads numbered 0..E[7]-1 bucket after bucket (E: running sums of
        // the buckets' extra ids), and id t's bucket and slot selected from
        // E and b by compares — a batch's QB id loads issue together, with
        // no dependent LDS read per id
        int32_t E[8];
        int32_t e = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            e += c[k] > WIDE_HEAD_IDS ? c[k] - WIDE_HEAD_IDS : 0;
            E[k] = e;
        }
        uint32_t tjn[QB];
        auto load_ids = [&](int32_t t0) {
#pragma unroll
            for (int u = 0; u < QB; ++u) {
                const int32_t t = t0 + u;
                uint32_t bk = b[7];
                int32_t base = E[6];
#pragma unroll
                for (int k = 6; k >= 0; --k)
                    if (t < E[k]) { bk = b[k]; base = k ? E[k - 1] : 0; }
                tjn[u] = t < e ? xld(slot_word(p.cur, bk, t - base + WIDE_HEAD_IDS, rl)) : (uint32_t)i;
            }
        };
        load_ids(0);
#pragma unroll 1
        for (int32_t t0 = 0; t0 < e; t0 += QB) {
            uint32_t tj[QB];
#pragma unroll
            for (int u = 0; u < QB; ++u) tj[u] = tjn[u];
            Snap<T> sn[QB];
#pragma unroll
            for (int u = 0; u < QB; ++u) {
                sn[u] = Snap<T>{x.x, x.y, x.z, T(0)};
                if ((tj[u] & ~BOX_FLAG) != (uint32_t)i) sn[u] = xld(p.snap_cur + CHK(tj[u] & ~BOX_FLAG, p.n_global));
            }
            if (t0 + QB < e) load_ids(t0 + QB);
#pragma unroll
            for (int u = 0; u < QB; ++u)
                if (t0 + u < e && hit(tj[u], sn[u])) append((int32_t)(tj[u] & ~BOX_FLAG), sn[u]);
        }
    }
    if (RB_WIDE_MORE && spm) {
#pragma unroll
        for (int k = 0; k < 8; ++k) s_cand[k * NB + tid] = b[k];
    }
#else
    if (RB_WIDE_MORE && more) {
        // buckets of 7+ bodies: the remaining ids from their lines, QB at a
        // time.  Rare, so kept compact: the buckets and counts go to the
        // lane's LDS column (s_cand is free now) and the loop over them is
        // not unrolled (unrolled, this path was 132 KB of the kernel's 194 KB)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            s_cand[k * NB + tid] = b[k];
            s_cand[(8 + k) * NB + tid] = (uint32_t)c[k];
        }
        auto test = [&](const uint32_t (&tj)[QB], const Snap<T> (&sn)[QB], int s0, int32_t ck) {
#pragma unroll
            for (int u = 0; u < QB; ++u)
                if (s0 + u < ck && hit(tj[u], sn[u])) {
                    append((int32_t)(tj[u] & ~BOX_FLAG), sn[u]);
                }
        };
        auto gather = [&](const uint32_t (&tj)[QB], Snap<T> (&sn)[QB]) {
#pragma unroll
            for (int u = 0; u < QB; ++u) {
                sn[u] = Snap<T>{x.x, x.y, x.z, T(0)};
                if ((tj[u] & ~BOX_FLAG) != (uint32_t)i) sn[u] = xld(p.snap_cur + CHK(tj[u] & ~BOX_FLAG, p.n_global));
            }
        };
#if RB_WIDE_PIPE
        // Software-pipelined, and batched across buckets: a batch takes the
        // next QB ids past the heads of whichever buckets still have some
        // (padding: the body itself, which never hits), and the ids of the
        // next batch load under the current batch's snapshots — a crowded
        // neighbourhood (C4's pile-ups: buckets of 7-30 ids) costs one
        // dependent round trip per QB candidates, not one or two per bucket
        int k = 0, s = WIDE_HEAD_IDS;
        uint32_t tjn[QB];
        auto load_ids = [&]() -> bool {           // the next batch's ids from cursor (k, s)
            bool any = false;
#pragma unroll
            for (int u = 0; u < QB; ++u) {
                while (k < 8 && s >= (int32_t)s_cand[(8 + k) * NB + tid]) { ++k; s = WIDE_HEAD_IDS; }
                tjn[u] = (uint32_t)i;
                if (k < 8) {
                    tjn[u] = xld(slot_word(p.cur, s_cand[k * NB + tid], s, rl));
                    ++s;
                    any = true;
                }
            }
            return any;
        };
        bool have = load_ids();
#pragma unroll 1
        while (have) {
            uint32_t tj[QB];
#pragma unroll
            for (int u = 0; u < QB; ++u) tj[u] = tjn[u];
            Snap<T> sn[QB];
            gather(tj, sn);
            have = load_ids();
            test(tj, sn, 0, QB);
        }
#else
#pragma unroll 1
        for (int k = 0; k < 8; ++k) {
            const uint32_t bk = s_cand[k * NB + tid];
            const int32_t ck = (int32_t)s_cand[(8 + k) * NB + tid];
#pragma unroll 1
            for (int s0 = WIDE_HEAD_IDS; s0 < ck; s0 += QB) {
                uint32_t tj[QB];
                Snap<T> sn[QB];
#pragma unroll
                for (int u = 0; u < QB; ++u)
                    tj[u] = s0 + u < ck ? xld(slot_word(p.cur, bk, s0 + u, rl)) : (uint32_t)i;
                gather(tj, sn);
                test(tj, sn, s0, ck);
            }
        }
#endif
    }
#endif
    if (RB_WIDE_MORE && spm) {                        // rarer: ids past full buckets (a spilled
#pragma unroll 1                                      // bucket is a 7+ one: its index is stashed)
        for (int k = 0; k < 8; ++k) {
            if (!((spm >> k) & 1u)) continue;
            spill_scan(p.cur, gen, s_cand[k * NB + tid], [&](uint32_t t) {
                const uint32_t j = t & ~BOX_FLAG;
                if (j == (uint32_t)i) return;
                const Snap<T> sn = xld(p.snap_cur + CHK(j, p.n_global));
                if (!hit(t, sn)) return;
                append((int32_t)j, sn);
            });
        }
    }
    // the partners in ascending id (the reference's contact order; distinct
    // ids: the wide search visits every bucket once, and a body sits in one
    // bucket or the spill list).  Long lists (C4's pile-ups, up to 28) are
    // sorted in registers by a bitonic network; short ones by rank: each
    // one's rank = how many are smaller, written to the lane's s_cand
    // column, then back.  s_didx maps a sorted position to the discovery
    // index (the s_hpos slot).  (The rank loop unrolled over the list's
    // capacity measured slower: C4's pile-up 72.0 -> 87.7 us,
    // profiles/r04/rank_unroll_ab_c4.log)
    if (np_ > WIDE_RANK_MAX) {
        sort_partners_bitonic<MAXP>(s_id, RB_WIDE_LDSPOS ? s_didx : nullptr, NB, tid, np_, nh);
    } else if (np_ > 1) {
        for (int u = 0; u < np_; ++u) {
            const int32_t v = s_id[u * NB + tid];
            int r = 0;
            for (int q = 0; q < np_; ++q) r += s_id[q * NB + tid] < v ? 1 : 0;
            s_cand[r * NB + tid] = (uint32_t)v;
            if (RB_WIDE_LDSPOS) s_didx[r * NB + tid] = (uint8_t)u;
        }
        for (int u = 0; u < np_; ++u) s_id[u * NB + tid] = (int32_t)s_cand[u * NB + tid];
    } else if (RB_WIDE_LDSPOS && np_ == 1) {
        s_didx[tid] = 0;
    }
    STAMP(10);
    if (overflow) atomicOr(p.err, ERR_PARTNER_OVERFLOW);
    return np_;
}

}  // namespace rb
