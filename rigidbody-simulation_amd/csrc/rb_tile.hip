// rb_tile.hip — K-step tile blocks: temporal blocking of the reference step
// (DESIGN §4.1).
//
// The reference step is Jacobi across bodies (one mj_forward per step,
// multi_sphere_bounce.py:43, then the per-body loop :46-90): after K steps a
// body depends only on bodies that came within contact reach of it, or of a
// body that did, within those K steps.  So one workgroup can take a spatial
// tile plus a ghost band around it and step that whole set K times out of
// LDS and registers — no broadphase table, no per-step launch, no HBM
// round trips — and keep the results of its own tile, which are then
// bit-identical to K single steps.
//
// Exactness is proven per block, not assumed:
//   * every body gets a displacement bound S (per axis) for the block, from
//     its speed over the previous block; its neighbour list is every body
//     that can come within contact reach under both bounds;
//   * the ring just outside the band is loaded too ("outer": never stepped)
//     and starts tainted; a stepped body is tainted at step s+1 when a
//     tainted list member's bound box reaches it at step s (or a body beyond
//     the ring could); untainted bodies read only untainted neighbours;
//   * the owner of each body checks after every step that it stayed inside
//     its bound.
// The block is exact for as many steps as no owned body was tainted and no
// bound was left.  If that is fewer than the block ran, the last workgroup
// schedules a redo from the same start (same bounds and lists, fewer steps),
// which is then exact by construction.  Decisions depend only on the state,
// so runs are deterministic.
#include "rb_device.hpp"
#include "rb_internal.hpp"

// diagnostic build only (RB_TILE_STAMPS=1, scripts/tile_stamps.py): summed
// per-phase cycles of every workgroup that stepped, read by rb_diag_tile_stamps
#ifndef RB_TILE_STAMPS
#define RB_TILE_STAMPS 0
#endif
#if RB_TILE_STAMPS
__device__ unsigned long long rb_tile_stamp_sum[16];
#define TSTAMP(k)                                                                                  \
    do {                                                                                           \
        __syncthreads();                                                                           \
        if (threadIdx.x == 0) {                                                                    \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();                            \
            if (k) atomicAdd(&rb_tile_stamp_sum[k], t_ - ts_prev);                                 \
            ts_prev = t_;                                                                          \
        }                                                                                          \
    } while (0)
#else
#define TSTAMP(k) do {} while (0)
#endif

namespace rb {

namespace {

constexpr uint8_t T_NEVER = 255;       // taint step of an untainted body
constexpr float S_C1 = 1.25f;          // speed margin of the displacement bound
constexpr float S_EPS = 1e-4f;         // absolute slack of bounds and box tests (m)

__device__ __forceinline__ int f2o(float f) { const int i = __float_as_int(f); return i >= 0 ? i : i ^ 0x7fffffff; }
__device__ __forceinline__ float o2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

// Displacement bound of a body after s steps of a block, per axis:
//   S_d(s) = s a1 + s (s + 1) a2_d + eps,   a1 = 1.25 dt sig,
//   a2_d = dt^2 (|g_d| + 2 mu (1 + e) |g|) / 2
// sig is the body's top speed over the previous block; the acceleration
// term covers gravity and a friction kick of mu (1 + e) u_n per ground
// contact (collision.py:42-46; twice that as margin).  A body that leaves
// its bound only shortens the block (the owner checks after every step).
template <typename T> __device__ __forceinline__ float speed_term(const TileParams<T> &p, float sig) {
    return (float)p.dt * (S_C1 * sig);
}
template <typename T> __device__ __forceinline__ float accel_term(const TileParams<T> &p, int d) {
    const float gm = sqrtf((float)(p.g[0] * p.g[0] + p.g[1] * p.g[1] + p.g[2] * p.g[2]));
    const float a = fabsf((float)p.g[d]) + 2.0f * (float)p.mu * (1.0f + (float)p.e) * gm;
    return 0.5f * (float)p.dt * (float)p.dt * a;
}
__device__ __forceinline__ float bound_at(int s, float a1, float a2) {
    return (float)s * a1 + (float)(s * (s + 1)) * a2 + S_EPS;
}

template <typename T>
__device__ __forceinline__ int tile_x(const TileParams<T> &p, T x) {
    const T f = (x - p.ox) / p.tile;
    int i = f > T(0) ? (int)f : 0;                 // NaN -> 0
    return i < p.ntx ? i : p.ntx - 1;
}
template <typename T>
__device__ __forceinline__ int tile_y(const TileParams<T> &p, T y) {
    const T f = (y - p.oy) / p.tile;
    int i = f > T(0) ? (int)f : 0;
    return i < p.nty ? i : p.nty - 1;
}

template <typename T>
__device__ __forceinline__ int64_t bin_at(const TileParams<T> &p, int ph, int t, int slot) {
    return ((int64_t)ph * p.ntile + t) * p.cap + slot;
}

// a record, moved with 16-byte accesses
template <typename T> __device__ __forceinline__ TileRec<T> load_rec(const TileRec<T> *r) {
    constexpr int NV = sizeof(TileRec<T>) / 16;
    union { uint4 u[NV]; TileRec<T> rec; } a;
    const uint4 *s = reinterpret_cast<const uint4 *>(r);
#pragma unroll
    for (int k = 0; k < NV; ++k) a.u[k] = s[k];
    return a.rec;
}
template <typename T> __device__ __forceinline__ void store_rec(TileRec<T> *r, const TileRec<T> &v) {
    constexpr int NV = sizeof(TileRec<T>) / 16;
    union { uint4 u[NV]; TileRec<T> rec; } a;
    a.rec = v;
    uint4 *d = reinterpret_cast<uint4 *>(r);
#pragma unroll
    for (int k = 0; k < NV; ++k) d[k] = a.u[k];
}

// world-frame inverse inertia of the step-start orientation, on first use
// (collision.py:62; value-identical to evaluating it every step).  The
// principal inertia stays in LDS until then (fewer live registers).
template <typename T> struct InvI {
    const T *I;                        // &s_I[0][lane], stride NT
    int stride;
    const Q4<T> &q;
    bool have;
    M3<T> m;
    __device__ __forceinline__ const M3<T> &get() {
        if (!have) {
            m = np_inv3(inertia_world(V3<T>{I[0], I[stride], I[2 * stride]}, q));
            have = true;
        }
        return m;
    }
};

// one contact through the reference's skip rules, then K2 (rb_kernels.hip
// solve_contact)
template <typename T>
__device__ __forceinline__ void tile_contact(const TileParams<T> &p, const Contact<T> &con, V3<T> x, V3<T> n, T m,
                                             T k, InvI<T> &inv, V3<T> &v, V3<T> &w) {
    if (!(con.dist < T(0))) return;                 // collision.py:74
    if (absval(con.dist) < p.thr) return;           // collision.py:79-80
    const V3<T> r = {con.pos.x - x.x, con.pos.y - x.y, con.pos.z - x.z};
    T jn;
    V3<T> jt;
    if (impulse(k, v, w, r, n, p.e, p.mu, jn, jt)) apply(v, w, m, inv.get(), r, n, jn, jt);
}

}  // namespace

// ---- canonical state -> bins[0] (one lane per owned body) ------------------
template <typename T>
__global__ __launch_bounds__(256) void tile_gather_kernel(TileParams<T> p) {
    const int64_t l = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (l >= p.n_local) return;
    const int32_t id = p.lo + (int32_t)l;
    const Snap<T> sn = p.snap_in[id];
    if (!(absval(sn.x) < T(1e9) && absval(sn.y) < T(1e9) && absval(sn.z) < T(1e9))) {
        atomicOr(p.err, ERR_DOMAIN);
        return;
    }
    const int t = tile_y(p, sn.y) * p.ntx + tile_x(p, sn.x);
    const int slot = atomicAdd(p.count + t, 1);
    if (slot >= p.cap) {
        atomicOr(&p.ctl->acc_err, ERR_TILE);
        return;
    }
    const T *st = p.st_base;
    TileRec<T> r;
    r.x = sn.x; r.y = sn.y; r.z = sn.z;
    r.qw = st[l]; r.qx = st[p.S + l]; r.qy = st[2 * p.S + l]; r.qz = st[3 * p.S + l];
    r.vx = st[4 * p.S + l]; r.vy = st[5 * p.S + l]; r.vz = st[6 * p.S + l];
    r.wx = st[7 * p.S + l]; r.wy = st[8 * p.S + l]; r.wz = st[9 * p.S + l];
    r.m = p.cs.mass()[id]; r.ix = p.cs.ix()[id]; r.iy = p.cs.iy()[id]; r.iz = p.cs.iz()[id];
    r.r = p.cs.sx()[id];
    r.id = id;
    // no history yet: the current speed (a violated bound just shortens the
    // first block)
    r.sig = (float)sqroot(r.vx * r.vx + r.vy * r.vy + r.vz * r.vz) * 1.0001f;
    store_rec(p.rec + bin_at(p, 0, t, slot), r);
    atomicMax(&p.ctl->sig_max, __float_as_uint(r.sig));
}

// ---- bins[phase] -> canonical state (state rows, snapshot of the final step) --
template <typename T>
__global__ __launch_bounds__(256) void tile_scatter_kernel(TileParams<T> p) {
    const int t = blockIdx.x;
    const int ph = p.ctl->phase;
    const int n = min(p.count[ph * p.ntile + t], p.cap);
    Snap<T> *out = p.snap_out[(p.c0 + p.ctl->done) & 1];
    T *st = p.st_base;
    for (int slot = threadIdx.x; slot < n; slot += 256) {
        const TileRec<T> r = load_rec(p.rec + bin_at(p, ph, t, slot));
        const int64_t l = r.id - p.lo;
        st[l] = r.qw; st[p.S + l] = r.qx; st[2 * p.S + l] = r.qy; st[3 * p.S + l] = r.qz;
        st[4 * p.S + l] = r.vx; st[5 * p.S + l] = r.vy; st[6 * p.S + l] = r.vz;
        st[7 * p.S + l] = r.wx; st[8 * p.S + l] = r.wy; st[9 * p.S + l] = r.wz;
        out[r.id] = Snap<T>{r.x, r.y, r.z, r.r};
    }
}

// ---- one block: K steps of one tile ---------------------------------------
template <typename T, int NT>
__global__ __launch_bounds__(NT) void tile_block_kernel(TileParams<T> p) {
    constexpr int LC = NT + NT / 2;            // LDS entries: [0, NT) stepped, [NT, LC) outer ring
    constexpr int NW = NT / 64;
    constexpr int NQ = 16;                     // edge-distance classes of the stepped entries
    __shared__ Snap<T> s_pos[2][NT];           // positions of the stepped bodies (ping-pong by step)
    __shared__ T s_x0[3][LC];                  // block-start positions
    __shared__ float s_a1[LC];                 // speed term of the displacement bound (bound_at)
    __shared__ float s_r[LC];                  // radii (rounded up)
    __shared__ int32_t s_gid[LC];
    __shared__ T s_I[3][NT];                   // principal inertia of the stepped bodies
    __shared__ T s_mr[2][NT];                  // their mass and radius (LDS, not VGPRs)
    __shared__ float s_sn[NT];                 // their top speed over the block (the next block's bound)
    __shared__ uint8_t s_t[LC];                // step at which the entry is tainted (T_NEVER: never)
    __shared__ uint16_t s_list[NT][TILE_MAXL]; // neighbour lists (entry indices, ascending global id)
    __shared__ int32_t s_nc[NT];               // their lengths
    __shared__ int32_t s_misc[32];
    __shared__ T s_ring[4];                    // outer ring box x0 x1 y0 y1 (fp64 values: LDS, not VGPRs)
    __shared__ int32_t s_ctot[TILE_NCOL / 64];
    __shared__ int32_t s_q[NQ + 1];            // edge-distance class counts, then offsets
    __shared__ uint16_t s_fast[LC];            // fast entries (wave-parallel list scans)
    __shared__ T s_ro[LC - NT];                // exact radii of the outer entries (their step-0 contacts)
    // build-time aliases: load references over the lists; the unsorted
    // references and the column sort over s_pos[1]
    uint32_t *s_ref = reinterpret_cast<uint32_t *>(&s_list[0][0]);
    uint32_t *s_col = reinterpret_cast<uint32_t *>(&s_pos[1][0]);
    uint16_t *s_sorted = reinterpret_cast<uint16_t *>(s_col + TILE_NCOL);
    uint32_t *s_tmp = reinterpret_cast<uint32_t *>(&s_pos[1][0]);
    uint8_t *s_key = reinterpret_cast<uint8_t *>(s_tmp + NT);
    static_assert(sizeof(s_list) >= sizeof(uint32_t) * LC, "load references alias the lists");
    static_assert(sizeof(s_pos[1]) >= sizeof(uint32_t) * TILE_NCOL + sizeof(uint16_t) * LC, "column sort aliases s_pos[1]");
    static_assert(sizeof(s_pos[1]) >= 5 * NT, "unsorted references alias s_pos[1]");

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    TileCtl *ctl = p.ctl;
    const int k_run = ctl->k_run;
    if (k_run <= 0) return;                    // nothing left: a no-op block
#if RB_TILE_STAMPS
    unsigned long long ts_prev = 0;
#endif
    TSTAMP(0);
    const int k_s = ctl->k_s, ph = ctl->phase;
    const float sig_max = __uint_as_float(ctl->sig_max);

    // tiles of an XCD (blocks b = x mod 8) form one contiguous strip of rows
    uint32_t t;
    {
        const uint32_t nb = gridDim.x, b = blockIdx.x, q = nb / 8, r = nb % 8, x = b % 8;
        t = x * q + (x < r ? x : r) + b / 8;
    }
    const int tx = (int)t % p.ntx, ty = (int)t / p.ntx;
    constexpr T INF = T(1e30);
    const T rx0 = tx == 0 ? -INF : p.ox + tx * p.tile, rx1 = tx == p.ntx - 1 ? INF : p.ox + (tx + 1) * p.tile;
    const T ry0 = ty == 0 ? -INF : p.oy + ty * p.tile, ry1 = ty == p.nty - 1 ? INF : p.oy + (ty + 1) * p.tile;
    const T W = p.band;
    const T lx0 = rx0 - W, lx1 = rx1 + W, ly0 = ry0 - W, ly1 = ry1 + W;
    // bounds: a body beyond the outer ring moves at most bound_at(s, af, a2) per axis
    const float af = speed_term(p, sig_max);
    float a2[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) a2[d] = accel_term(p, d);
    const T Sfx = (T)bound_at(k_s, af, a2[0]), Sfy = (T)bound_at(k_s, af, a2[1]);
    const T M = T(2) * p.rmax + (Sfx > Sfy ? Sfx : Sfy) + T(S_EPS);
    const T ox0 = lx0 - M, ox1 = lx1 + M, oy0 = ly0 - M, oy1 = ly1 + M;
    if (tid < 32) s_misc[tid] = (tid == 4 || tid == 6) ? INT32_MAX : (tid == 5 || tid == 7) ? INT32_MIN : 0;
    if (tid == 2) s_misc[2] = (W + M + (Sfx > Sfy ? Sfx : Sfy) > p.tile) ? ERR_TILE : 0;   // ring within the 9 bins
    if (tid == 3) s_misc[3] = k_run;           // steps valid (min over owned bodies)
    if (tid == 4) { s_ring[0] = ox0; s_ring[1] = ox1; s_ring[2] = oy0; s_ring[3] = oy1; }
    if (tid <= NQ) s_q[tid] = 0;
    __syncthreads();

    // ---- 1. the 9 bins around the tile: band (loaded, may be stepped) and
    // outer (ring) entries.  Band entries are ordered by their distance from
    // the tile, nearest first: the far ones are stepped for fewer steps or
    // not at all (hop distances, below), so whole waves fall idle
    int pre[10];
    int binid[9];
    pre[0] = 0;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        const int bx = tx + j % 3 - 1, by = ty + j / 3 - 1;
        const bool ok = bx >= 0 && bx < p.ntx && by >= 0 && by < p.nty;
        binid[j] = ok ? by * p.ntx + bx : 0;
        const int cnt = ok ? p.count[ph * p.ntile + binid[j]] : 0;
        pre[j + 1] = pre[j] + (cnt < p.cap ? cnt : p.cap);
    }
    const T qinv = T(NQ) / W;
    for (int base = 0; base < pre[9]; base += 4 * NT) {
        T cx[4], cy[4];
        uint32_t cref[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int idx = base + u * NT + tid;
            // the last bin starting at or before idx (selects: no indexed private array)
            int b = binid[0], b0 = 0;
#pragma unroll
            for (int j = 1; j < 9; ++j)
                if (idx >= pre[j]) { b = binid[j]; b0 = pre[j]; }
            const uint32_t ref = (uint32_t)b * (uint32_t)p.cap + (uint32_t)(idx - b0);
            cref[u] = idx < pre[9] ? ref : 0xffffffffu;
            if (idx < pre[9]) {
                const TileRec<T> *r = p.rec + bin_at(p, ph, b, idx - b0);
                if constexpr (sizeof(T) == 8) {
                    const double2 xy = *reinterpret_cast<const double2 *>(r);
                    cx[u] = xy.x; cy[u] = xy.y;
                } else {
                    const float2 xy = *reinterpret_cast<const float2 *>(r);
                    cx[u] = xy.x; cy[u] = xy.y;
                }
            }
        }
        // classify, with one LDS atomic per wave and class (not per lane)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const bool have = cref[u] != 0xffffffffu;
            const T x = have ? cx[u] : T(0), y = have ? cy[u] : T(0);
            const bool fin = absval(x) < T(1e9) && absval(y) < T(1e9);
            if (have && !fin) atomicOr(p.err, ERR_DOMAIN);   // non-finite / runaway position (rb_grid.hpp cell_of)
            const bool isl = have && fin && x >= lx0 && x < lx1 && y >= ly0 && y < ly1;
            const bool iso = have && fin && !isl && x >= ox0 && x < ox1 && y >= oy0 && y < oy1;
            // distance from the owned rectangle (0 inside) in NQ classes
            const T dx = fmax(fmax(rx0 - x, x - rx1), T(0)), dy = fmax(fmax(ry0 - y, y - ry1), T(0));
            const T de = fmax(dx, dy);
            const int q = de * qinv < T(NQ - 1) ? (int)(de * qinv) : NQ - 1;
            const uint64_t bl = __ballot(isl), bo = __ballot(iso), lt = (1ull << lane) - 1ull;
            int bL = 0, bO = 0;
            if (lane == 0) {
                if (bl) bL = atomicAdd(&s_misc[0], __popcll(bl));
                if (bo) bO = atomicAdd(&s_misc[1], __popcll(bo));
            }
            bL = __shfl(bL, 0);
            bO = __shfl(bO, 0);
            if (isl) {
                const int e = bL + __popcll(bl & lt);
                if (e < NT) { s_tmp[e] = cref[u]; s_key[e] = (uint8_t)q; }
                else s_misc[2] = ERR_TILE;
            }
            if (iso) {
                const int o = bO + __popcll(bo & lt);
                if (o < LC - NT) s_ref[NT + o] = cref[u];
                else s_misc[2] = ERR_TILE;
            }
        }
    }
    __syncthreads();
    const int nl = s_misc[0] < NT ? s_misc[0] : NT, no = s_misc[1] < LC - NT ? s_misc[1] : LC - NT;
    // a tile over capacity (band or ring) steps nothing: the run stops and
    // the host resumes on the per-step kernels (no entry may be left unset)
    const bool over = s_misc[2] != 0;
    if (!over) {
    // the stored band entries in distance-class order (counted, scanned, placed)
    if (tid < nl) atomicAdd(&s_q[s_key[tid]], 1);
    __syncthreads();
    if (tid == 0) {
        int a = 0;
        for (int k = 0; k < NQ; ++k) { const int c = s_q[k]; s_q[k] = a; a += c; }
    }
    __syncthreads();
    if (tid < nl) s_ref[atomicAdd(&s_q[s_key[tid]], 1)] = s_tmp[tid];
    __syncthreads();
    TSTAMP(1);

    // ---- 2. records -> registers (stepped) and LDS (every entry)
    V3<T> x{}, v{}, w{};
    Q4<T> q{};
    bool own = false;
    const uint32_t nref = (uint32_t)p.ntile * (uint32_t)p.cap;
    if (tid < nl && s_ref[tid] >= nref) { s_ref[tid] = 0; atomicOr(&ctl->acc_err, ERR_TILE); }   // (never: defensive)
    if (tid < no && s_ref[NT + tid] >= nref) { s_ref[NT + tid] = 0; atomicOr(&ctl->acc_err, ERR_TILE); }
    if (tid < nl) {
        const uint32_t ref = s_ref[tid];
        const TileRec<T> r = load_rec(p.rec + bin_at(p, ph, (int)(ref / (uint32_t)p.cap), (int)(ref % (uint32_t)p.cap)));
        x = {r.x, r.y, r.z};
        q = {r.qw, r.qx, r.qy, r.qz};
        v = {r.vx, r.vy, r.vz};
        w = {r.wx, r.wy, r.wz};
        s_mr[0][tid] = r.m;
        s_I[0][tid] = r.ix;
        s_I[1][tid] = r.iy;
        s_I[2][tid] = r.iz;
        s_mr[1][tid] = r.r;                    // spheres only: the bound is the radius
        own = tile_x(p, x.x) == tx && tile_y(p, x.y) == ty;
        s_pos[0][tid] = Snap<T>{x.x, x.y, x.z, r.r};
        s_x0[0][tid] = x.x; s_x0[1][tid] = x.y; s_x0[2][tid] = x.z;
        s_a1[tid] = speed_term(p, r.sig);
        s_r[tid] = (float)r.r * 1.000001f;
        s_gid[tid] = r.id;
        s_t[tid] = T_NEVER;
        s_sn[tid] = (float)sqroot(v.x * v.x + v.y * v.y + v.z * v.z);
        if (own) atomicAdd(&s_misc[12], 1);
    }
    if (tid < no) {
        const int e = NT + tid;
        const uint32_t ref = s_ref[e];
        const TileRec<T> *r = p.rec + bin_at(p, ph, (int)(ref / (uint32_t)p.cap), (int)(ref % (uint32_t)p.cap));
        s_x0[0][e] = r->x; s_x0[1][e] = r->y; s_x0[2][e] = r->z;
        s_a1[e] = speed_term(p, r->sig);
        s_ro[tid] = r->r;
        s_r[e] = (float)r->r * 1.000001f;
        s_gid[e] = r->id;
        s_t[e] = 1;                            // outer: exact at the block start only
    }
    // column grid extent: the entries' xy box; the bounds' largest and mean speed terms
    {
        float bx0 = 3e38f, bx1 = -3e38f, by0 = 3e38f, by1 = -3e38f, smax = 0.f, asum = 0.f;
        if (tid < nl) {
            bx0 = bx1 = (float)x.x; by0 = by1 = (float)x.y;
            smax = asum = s_a1[tid];
        }
        if (tid < no) {
            const float ex = (float)s_x0[0][NT + tid], ey = (float)s_x0[1][NT + tid];
            bx0 = fminf(bx0, ex); bx1 = fmaxf(bx1, ex); by0 = fminf(by0, ey); by1 = fmaxf(by1, ey);
            smax = fmaxf(smax, s_a1[NT + tid]);
            asum += s_a1[NT + tid];
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            bx0 = fminf(bx0, __shfl_xor(bx0, o)); bx1 = fmaxf(bx1, __shfl_xor(bx1, o));
            by0 = fminf(by0, __shfl_xor(by0, o)); by1 = fmaxf(by1, __shfl_xor(by1, o));
            smax = fmaxf(smax, __shfl_xor(smax, o));
            asum += __shfl_xor(asum, o);
        }
        if (lane == 0) {
            atomicMin(&s_misc[4], f2o(bx0)); atomicMax(&s_misc[5], f2o(bx1));
            atomicMin(&s_misc[6], f2o(by0)); atomicMax(&s_misc[7], f2o(by1));
            atomicMax(&s_misc[8], f2o(smax));
            atomicAdd(reinterpret_cast<float *>(&s_misc[13]), asum);
        }
    }
    __syncthreads();
    TSTAMP(2);
    int my_valid = k_run;
    int disp_bad = 0;
    if (s_misc[12] > 0) {                      // (uniform) a tile with bodies to step
    // ---- 3. neighbour lists: counting sort of the entries by xy column.
    // A pair is a candidate when, per axis, its block-start separation is
    // below both radii plus both displacement bounds at the block horizon.
    // Columns are sized for the slow entries (speed term at most 3 x the
    // mean); a slow body scans its 3 x 3 columns for slow candidates; a fast
    // entry is scanned by a whole wave as far as its bound reaches, and
    // enters itself in the lists of the slow bodies it finds.  Lists are
    // then sorted by global id.
    const float gx0 = o2f(s_misc[4]), gy0 = o2f(s_misc[6]);
    const float gx1 = o2f(s_misc[5]), gy1 = o2f(s_misc[7]);
    const float a2xy = a2[0] > a2[1] ? a2[0] : a2[1];
    const float a1_max = o2f(s_misc[8]);
    const float a1_thr = fminf(a1_max, 3.0f * __int_as_float(s_misc[13]) / (float)(nl + no > 0 ? nl + no : 1));
    const float r2 = 2.0f * (float)p.rmax * 1.000001f;
    float cs = r2 + 2.0f * bound_at(k_s, a1_thr, a2xy) + 2.0f * S_EPS;
    int ncx = (int)((gx1 - gx0) / cs) + 1, ncy = (int)((gy1 - gy0) / cs) + 1;
    while ((int64_t)ncx * ncy > TILE_NCOL) {
        cs *= 1.25f;
        ncx = (int)((gx1 - gx0) / cs) + 1;
        ncy = (int)((gy1 - gy0) / cs) + 1;
    }
    const float smax_all = bound_at(k_s, a1_max, a2xy);
    auto col_of = [&](float ex, float ey) {
        int cx = (int)((ex - gx0) / cs), cy = (int)((ey - gy0) / cs);
        cx = cx < 0 ? 0 : cx >= ncx ? ncx - 1 : cx;
        cy = cy < 0 ? 0 : cy >= ncy ? ncy - 1 : cy;
        return cy * ncx + cx;
    };
    for (int c = tid; c < TILE_NCOL; c += NT) s_col[c] = 0;
    s_nc[tid] = 0;
    __syncthreads();
    int col_l = -1, col_o = -1;
    if (tid < nl) { col_l = col_of((float)x.x, (float)x.y); atomicAdd(&s_col[col_l], 1u); }
    if (tid < no) { col_o = col_of((float)s_x0[0][NT + tid], (float)s_x0[1][NT + tid]); atomicAdd(&s_col[col_o], 1u); }
    // fast entries, for the wave-parallel scans
    if (tid < nl && s_a1[tid] > a1_thr) s_fast[atomicAdd(&s_misc[14], 1)] = (uint16_t)tid;
    if (tid < no && s_a1[NT + tid] > a1_thr) s_fast[atomicAdd(&s_misc[14], 1)] = (uint16_t)(NT + tid);
    __syncthreads();
    // exclusive scan of the column counts (chunks of 64 by wave, then the chunk totals)
    for (int ch = wave; ch < TILE_NCOL / 64; ch += NW) {
        const int c = ch * 64 + lane;
        const uint32_t n0 = s_col[c];
        uint32_t s = n0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(s, o);
            if (lane >= o) s += u;
        }
        s_col[c] = s - n0;
        if (lane == 63) s_ctot[ch] = (int32_t)s;
    }
    __syncthreads();
    if (tid == 0) {
        int32_t a = 0;
        for (int ch = 0; ch < TILE_NCOL / 64; ++ch) { const int32_t n0 = s_ctot[ch]; s_ctot[ch] = a; a += n0; }
    }
    __syncthreads();
    for (int c = tid; c < TILE_NCOL; c += NT) s_col[c] += (uint32_t)s_ctot[c >> 6];
    __syncthreads();
    if (col_l >= 0) s_sorted[atomicAdd(&s_col[col_l], 1u)] = (uint16_t)tid;
    if (col_o >= 0) s_sorted[atomicAdd(&s_col[col_o], 1u)] = (uint16_t)(NT + tid);
    __syncthreads();
    TSTAMP(12);
    // now s_col[c] = end of column c = start of column c + 1
    auto append = [&](int owner, int mi) {
        const int k = atomicAdd(&s_nc[owner], 1);
        if (k < TILE_MAXL) s_list[owner][k] = (uint16_t)mi;
    };
    // the pair test of entry e against candidate mi (e's bounds precomputed)
    auto pair = [&](T ex, T ey, T ez, float ra, float sa0, float sa1, float sa2, int mi) {
        const float b1 = s_a1[mi];
        const float rr = ra + s_r[mi] + S_EPS;
        return fabsf((float)(ex - s_x0[0][mi])) < rr + sa0 + bound_at(k_s, b1, a2[0]) &&
               fabsf((float)(ey - s_x0[1][mi])) < rr + sa1 + bound_at(k_s, b1, a2[1]) &&
               fabsf((float)(ez - s_x0[2][mi])) < rr + sa2 + bound_at(k_s, b1, a2[2]);
    };
    if (tid < nl && s_a1[tid] <= a1_thr) {     // a slow body: its 3 x 3 columns, slow candidates
        const float ra = s_r[tid], a1 = s_a1[tid];
        const float sa0 = bound_at(k_s, a1, a2[0]), sa1 = bound_at(k_s, a1, a2[1]), sa2 = bound_at(k_s, a1, a2[2]);
        const int mcx = col_l % ncx, mcy = col_l / ncx;
        for (int yy = max(mcy - 1, 0); yy <= min(mcy + 1, ncy - 1); ++yy) {
            const int c0 = yy * ncx + max(mcx - 1, 0), c1 = yy * ncx + min(mcx + 1, ncx - 1);
            const uint32_t u0 = c0 ? s_col[c0 - 1] : 0u, u1 = s_col[c1];
            for (uint32_t u = u0; u < u1; ++u) {
                const int mi = s_sorted[u];
                if (mi == tid || s_a1[mi] > a1_thr) continue;   // fast ones enter themselves
                if (pair(x.x, x.y, x.z, ra, sa0, sa1, sa2, mi)) append(tid, mi);
            }
        }
    }
    // fast entries: one wave each, lanes over the candidates of each row
    for (int fi = wave; fi < s_misc[14]; fi += NW) {
        const int e = s_fast[fi];
        const T ex = s_x0[0][e], ey = s_x0[1][e], ez = s_x0[2][e];
        const float ra = s_r[e], a1 = s_a1[e];
        const float sa0 = bound_at(k_s, a1, a2[0]), sa1 = bound_at(k_s, a1, a2[1]), sa2 = bound_at(k_s, a1, a2[2]);
        const int col = col_of((float)ex, (float)ey), mcx = col % ncx, mcy = col / ncx;
        const int reach = (int)((r2 + bound_at(k_s, a1, a2xy) + smax_all + 2.0f * S_EPS) / cs) + 1;
        // the rows' candidate ranges (contiguous in s_sorted), 8 rows at a
        // time, flattened over the wave's lanes
        const int ya = max(mcy - reach, 0), yb = min(mcy + reach, ncy - 1);
        const int xa = max(mcx - reach, 0), xb = min(mcx + reach, ncx - 1);
        for (int y0 = ya; y0 <= yb; y0 += 8) {
            uint32_t ru0[8], rpre[9];
            rpre[0] = 0;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int yy = y0 + r;
                const int c0 = yy * ncx + xa, c1 = yy * ncx + xb;
                const uint32_t u0 = yy <= yb ? (c0 ? s_col[c0 - 1] : 0u) : 0u;
                const uint32_t u1 = yy <= yb ? s_col[c1] : 0u;
                ru0[r] = u0;
                rpre[r + 1] = rpre[r] + (u1 - u0);
            }
            for (uint32_t idx = lane; idx < rpre[8]; idx += 64) {
                uint32_t u = ru0[0] + idx;
#pragma unroll
                for (int r = 1; r < 8; ++r)
                    if (idx >= rpre[r]) u = ru0[r] + (idx - rpre[r]);
                const int mi = s_sorted[u];
                if (mi == e || !pair(ex, ey, ez, ra, sa0, sa1, sa2, mi)) continue;
                if (e < NT) append(e, mi);
                if (mi < NT && s_a1[mi] <= a1_thr) append(mi, e);   // a fast candidate lists e itself
            }
        }
    }
    __syncthreads();
    TSTAMP(13);
    if (tid < nl) {
        int n = s_nc[tid];
        if (n > TILE_MAXL) { n = TILE_MAXL; s_t[tid] = 1; }   // list incomplete: exact at the block start only
        // insertion sort by global id (the canonical partner order)
        for (int i = 1; i < n; ++i) {
            const uint16_t mi = s_list[tid][i];
            const int32_t g = s_gid[mi];
            int k = i;
            while (k > 0 && s_gid[s_list[tid][k - 1]] > g) { s_list[tid][k] = s_list[tid][k - 1]; --k; }
            s_list[tid][k] = mi;
        }
        s_nc[tid] = n;
    }
    __syncthreads();

    // hop distance of every band body from the tile's own bodies over the
    // lists (capped at k_run): a body d hops out is needed exact only
    // through step k_run - d, so it retires there (its taint step), and a
    // body k_run hops out is not stepped at all.  Lists are symmetric, so a
    // neighbour retires at most one step before a body that still needs it.
    int hop = k_run;
    if (tid < nl && own) hop = 0;
    __shared__ uint8_t s_hop[NT];
    if (tid < NT) s_hop[tid] = (uint8_t)(tid < nl ? hop : k_run);
    __syncthreads();
    for (int it = 0; it < k_run; ++it) {
        if (tid < nl && hop > 0) {
            const int n = s_nc[tid];
            for (int k = 0; k < n; ++k) {
                const int mi = s_list[tid][k];
                if (mi < NT) hop = min(hop, (int)s_hop[mi] + 1);
            }
            s_hop[tid] = (uint8_t)hop;
        }
        __syncthreads();
    }
    if (tid < nl) {
        const int need = k_run - hop;          // steps this body must be exact for
        const int t0 = s_t[tid];               // 1 after a list overflow
        s_t[tid] = (uint8_t)min(min(t0, need + 1), (int)T_NEVER);
        if (own && t0 <= 1) my_valid = 0;      // an owned body whose list overflowed
    }
    __syncthreads();

    TSTAMP(3);
    // ---- 4. K steps
    for (int s = 0; s < k_run; ++s) {
        const int cur = s & 1;
        // stepped: still needed after this step (t = the first step whose
        // position is not known exact) and not tainted below
        if (tid < nl && s_t[tid] > s + 1) {
#if RB_TILE_STAMPS
            atomicAdd(&rb_tile_stamp_sum[14], 1ull);                  // active lanes x steps
            if (lane == __builtin_ctzll(__ballot(1))) atomicAdd(&rb_tile_stamp_sum[15], 1ull);   // active waves x steps
#endif
            const T rad = s_mr[1][tid];
            const int nlist = s_nc[tid];
            // a body beyond the ring (moved at most its bound) in reach?
            const T fx = (T)bound_at(s, af, a2[0]) + rad + p.rmax, fy = (T)bound_at(s, af, a2[1]) + rad + p.rmax;
            bool taint = (x.x - s_ring[0] < fx) || (s_ring[1] - x.x < fx) || (x.y - s_ring[2] < fy) ||
                         (s_ring[3] - x.y < fy);
            // each batch of 4 neighbours' taint step and position together:
            // tainted ones are tested against their bound box, the others
            // decide contact now (positions only), so the solves below walk
            // the hits alone
            uint32_t hits = 0;
#pragma unroll 1
            for (int b0 = 0; b0 < TILE_MAXL; b0 += 4) {
                if (b0 < nlist) {
                    int mi[4];
                    uint8_t tt[4];
                    Snap<T> pe[4];
                    const uint2 lw = *reinterpret_cast<const uint2 *>(&s_list[tid][b0]);   // 4 entries, one read
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        mi[u] = (int)(((u < 2 ? lw.x : lw.y) >> (16 * (u & 1))) & 0xffffu);
                        if (b0 + u < nlist) {
                            tt[u] = s_t[mi[u]];
                            if (mi[u] < NT) pe[u] = s_pos[cur][mi[u]];
                            else pe[u] = Snap<T>{s_x0[0][mi[u]], s_x0[1][mi[u]], s_x0[2][mi[u]], s_ro[mi[u] - NT]};
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        if (b0 + u >= nlist) continue;
                        if (tt[u] <= s) {
                            // a tainted neighbour: could its true position (within
                            // its bound of step s) reach this body?
                            T g2 = T(0);
                            const float b1 = s_a1[mi[u]];
#pragma unroll
                            for (int d = 0; d < 3; ++d) {
                                const T xd = d == 0 ? x.x : d == 1 ? x.y : x.z;
                                T gap = absval(xd - s_x0[d][mi[u]]) - (T)bound_at(s, b1, a2[d]);
                                gap = gap > T(0) ? gap : T(0);
                                g2 += gap * gap;
                            }
                            const T rr = rad + (T)s_r[mi[u]] + T(S_EPS);
                            taint = taint || g2 < rr * rr;
                        } else if (sphere_sphere_hit(x, rad, V3<T>{pe[u].x, pe[u].y, pe[u].z}, pe[u].r)) {
                            hits |= 1u << (b0 + u);
                        }
                    }
                }
            }
            if (taint) {
                s_t[tid] = (uint8_t)(s + 1);
                if (own && my_valid > s) my_valid = s;
            } else {
                // one reference step (rb_kernels.hip body_update, same operation order)
                const T m = s_mr[0][tid];
                InvI<T> inv{&s_I[0][tid], NT, q, false, {}};
                {
                    const V3<T> F = {m * p.g[0], m * p.g[1], m * p.g[2]};      // collision.py:66-69
                    v = {v.x + (F.x / m) * p.dt, v.y + (F.y / m) * p.dt, v.z + (F.z / m) * p.dt};
                }
                const T kk = impulse_k(m);
                // plane contacts (plane order), then the partner hits in list
                // (= ascending id) order: one solve site for both
                const int npl = p.n_planes;
                int k = 0;
                for (;;) {
                    Contact<T> con;
                    V3<T> n;
                    if (k < npl) {
                        const V3<T> pn = {p.pn[k][0], p.pn[k][1], p.pn[k][2]};
                        const V3<T> pp = {p.pp[k][0], p.pp[k][1], p.pp[k][2]};
                        ++k;
                        if (!plane_sphere(pn, pp, x, rad, con)) continue;
                        n = con.frame;
                    } else {
                        if (!hits) break;
                        const int kb = __builtin_ctz(hits);
                        hits &= hits - 1u;
                        const int mi = s_list[tid][kb];
                        const Snap<T> pe = mi < NT ? s_pos[cur][mi]
                                                   : Snap<T>{s_x0[0][mi], s_x0[1][mi], s_x0[2][mi], s_ro[mi - NT]};
                        const V3<T> cj = {pe.x, pe.y, pe.z};
                        if (s_gid[tid] < s_gid[mi]) {         // this body is geom1
                            sphere_sphere(x, rad, cj, pe.r, con);
                            n = p.oriented ? V3<T>{-con.frame.x, -con.frame.y, -con.frame.z} : con.frame;
                        } else {
                            sphere_sphere(cj, pe.r, x, rad, con);
                            n = con.frame;
                        }
                    }
                    tile_contact(p, con, x, n, m, kk, inv, v, w);
                }
                // K3 (collision.py:90-95)
                x = {x.x + v.x * p.dt, x.y + v.y * p.dt, x.z + v.z * p.dt};
                const Q4<T> res = mj_mulquat(Q4<T>{T(0), w.x, w.y, w.z}, q);
                Q4<T> qn = {q.w + (T(0.5) * res.w) * p.dt, q.x + (T(0.5) * res.x) * p.dt,
                            q.y + (T(0.5) * res.y) * p.dt, q.z + (T(0.5) * res.z) * p.dt};
                const T nq = sqroot(fmadd(qn.z, qn.z, fmadd(qn.y, qn.y, fmadd(qn.x, qn.x, qn.w * qn.w))));
                q = {qn.w / nq, qn.x / nq, qn.y / nq, qn.z / nq};
                s_pos[cur ^ 1][tid] = Snap<T>{x.x, x.y, x.z, rad};
                if (own) {
                    const float a1 = s_a1[tid];
                    const bool out = absval(x.x - s_x0[0][tid]) > (T)bound_at(s + 1, a1, a2[0]) ||
                                     absval(x.y - s_x0[1][tid]) > (T)bound_at(s + 1, a1, a2[1]) ||
                                     absval(x.z - s_x0[2][tid]) > (T)bound_at(s + 1, a1, a2[2]);
                    if (out && my_valid > s + 1) { my_valid = s + 1; disp_bad = 1; }
                    s_sn[tid] = fmaxf(s_sn[tid], (float)sqroot(v.x * v.x + v.y * v.y + v.z * v.z));
                }
            }
        }
        __syncthreads();
    }
    }

    TSTAMP(4);
    // ---- 5. owned bodies -> bins[1 - phase][t]; validity and the new speed bound
    {
        int mv = (tid < nl && own) ? my_valid : k_run;
        int db = disp_bad;
        float sg = (tid < nl && own) ? s_sn[tid] : 0.f;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            mv = min(mv, __shfl_xor(mv, o));
            db |= __shfl_xor(db, o);
            sg = fmaxf(sg, __shfl_xor(sg, o));
        }
        if (lane == 0) {
            atomicMin(&s_misc[3], mv);
            atomicOr(&s_misc[9], db);
            atomicMax(&s_misc[10], __float_as_int(sg));
        }
    }
    const bool wr = tid < nl && own;
    const uint64_t bal = __ballot(wr);
    int slot = 0;
    {
        // wave offsets in wave order
        __shared__ int32_t s_wc[NW + 1];
        if (lane == 0) s_wc[wave] = __popcll(bal);
        __syncthreads();
        if (tid == 0) {
            int a = 0;
            for (int k = 0; k < NW; ++k) { const int n0 = s_wc[k]; s_wc[k] = a; a += n0; }
            s_wc[NW] = a;
        }
        __syncthreads();
        slot = s_wc[wave] + __popcll(bal & ((1ull << lane) - 1ull));
        if (tid == 0) {
            if (s_wc[NW] > p.cap) atomicOr(&ctl->acc_err, ERR_TILE);
            p.count[(1 - ph) * p.ntile + (int)t] = s_wc[NW] < p.cap ? s_wc[NW] : p.cap;
        }
    }
    if (wr && !(absval(x.x) < T(1e9) && absval(x.y) < T(1e9) && absval(x.z) < T(1e9))) atomicOr(p.err, ERR_DOMAIN);
    if (wr && slot < p.cap) {
        TileRec<T> r;
        r.x = x.x; r.y = x.y; r.z = x.z;
        r.qw = q.w; r.qx = q.x; r.qy = q.y; r.qz = q.z;
        r.vx = v.x; r.vy = v.y; r.vz = v.z;
        r.wx = w.x; r.wy = w.y; r.wz = w.z;
        r.m = s_mr[0][tid]; r.ix = s_I[0][tid]; r.iy = s_I[1][tid]; r.iz = s_I[2][tid]; r.r = s_mr[1][tid];
        r.id = s_gid[tid];
        r.sig = s_sn[tid] * 1.0001f;
        store_rec(p.rec + bin_at(p, 1 - ph, (int)t, slot), r);
    }

    TSTAMP(5);
    } else if (tid == 0) {                     // capacity: the run falls back
        atomicOr(&ctl->acc_err, s_misc[2]);
        s_misc[3] = 0;
    }
#if RB_TILE_STAMPS
    if (tid == 0) { atomicAdd(&rb_tile_stamp_sum[8], 1ull); atomicAdd(&rb_tile_stamp_sum[9], (unsigned long long)k_run);
                    atomicAdd(&rb_tile_stamp_sum[10], (unsigned long long)nl); atomicAdd(&rb_tile_stamp_sum[11], (unsigned long long)no); }
#endif
    // ---- 6. the last workgroup closes the block: commit, or redo shorter
    if (tid == 0) {
        atomicMin(&ctl->acc_valid, s_misc[3]);
        atomicMax(&ctl->acc_sig, (uint32_t)s_misc[10]);
        if (s_misc[9]) atomicOr(&ctl->acc_disp, 1);
        __threadfence();
        const uint32_t d = atomicAdd(&ctl->acc_done, 1u);
        if (d == gridDim.x - 1) {
            __threadfence();
            const int valid = atomicAdd(&ctl->acc_valid, 0);
            const int err = atomicAdd(&ctl->acc_err, 0);
            const uint32_t sg = atomicAdd(&ctl->acc_sig, 0u);
            const int disp = atomicAdd(&ctl->acc_disp, 0);
            ctl->blocks += 1;
            if (err) {
                ctl->err |= err;
                ctl->k_run = 0;                // stop: the host resumes from `done`
            } else if (valid >= k_run) {       // commit
                ctl->done += k_run;
                ctl->phase = 1 - ph;
                ctl->sig_max = sg;
                // the next horizon: a redone block's length; after 4 clean
                // blocks in a row, one step longer (a failed probe costs a block)
                int kn = k_run;
                if (k_run == k_s) {
                    ctl->streak += 1;
                    if (ctl->streak >= 4 && k_s < p.kmax) { kn = k_s + 1; ctl->streak = 0; }
                } else {
                    ctl->streak = 0;
                }
                ctl->k_plan = kn;
                ctl->k_s = kn;
                const int64_t left = ctl->target - ctl->done;
                ctl->k_run = (int)(left < kn ? left : kn);
            } else if (valid >= 1) {           // redo the first `valid` steps (exact by construction)
                ctl->k_run = valid;
                if (disp) ctl->redo_disp += 1; else ctl->redo_taint += 1;
            } else if (k_s > 1) {              // not even one step: rebuild at horizon 1
                ctl->k_s = 1;
                ctl->k_run = 1;
                ctl->restart += 1;
            } else {
                ctl->err |= ERR_TILE;          // the band is too thin for this scene
                ctl->k_run = 0;
            }
            ctl->acc_valid = 1 << 30;
            ctl->acc_err = 0;
            ctl->acc_sig = 0u;
            ctl->acc_disp = 0;
            ctl->acc_done = 0u;
        }
    }
}

#if RB_TILE_STAMPS
extern "C" int rb_diag_tile_stamps(unsigned long long *out, int reset) {
    int r = (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(rb_tile_stamp_sum), sizeof(unsigned long long) * 16);
    if (reset) {
        unsigned long long z[16] = {};
        r |= (int)hipMemcpyToSymbol(HIP_SYMBOL(rb_tile_stamp_sum), z, sizeof z);
    }
    return r;
}
#endif

template <typename T> hipError_t launch_tile_gather(const TileParams<T> &p, hipStream_t s) {
    if (p.n_local <= 0) return hipSuccess;
    hipLaunchKernelGGL((tile_gather_kernel<T>), dim3((unsigned)((p.n_local + 255) / 256)), dim3(256), 0, s, p);
    return hipGetLastError();
}
template <typename T> hipError_t launch_tile_block(const TileParams<T> &p, int nt, hipStream_t s) {
    // fp64: 512 threads (206 VGPRs, 2 waves per SIMD, no spill); fp32: 768
    if constexpr (sizeof(T) == 8) {
        if (nt == 256) hipLaunchKernelGGL((tile_block_kernel<T, 256>), dim3((unsigned)p.ntile), dim3(256), 0, s, p);
        else if (nt == 512) hipLaunchKernelGGL((tile_block_kernel<T, 512>), dim3((unsigned)p.ntile), dim3(512), 0, s, p);
        else return hipErrorInvalidValue;
    } else {
        if (nt != 768) return hipErrorInvalidValue;
        hipLaunchKernelGGL((tile_block_kernel<T, 768>), dim3((unsigned)p.ntile), dim3(768), 0, s, p);
    }
    return hipGetLastError();
}
template <typename T> hipError_t launch_tile_scatter(const TileParams<T> &p, hipStream_t s) {
    hipLaunchKernelGGL((tile_scatter_kernel<T>), dim3((unsigned)p.ntile), dim3(256), 0, s, p);
    return hipGetLastError();
}

template hipError_t launch_tile_gather<double>(const TileParams<double> &, hipStream_t);
template hipError_t launch_tile_block<double>(const TileParams<double> &, int, hipStream_t);
template hipError_t launch_tile_scatter<double>(const TileParams<double> &, hipStream_t);
template hipError_t launch_tile_gather<float>(const TileParams<float> &, hipStream_t);
template hipError_t launch_tile_block<float>(const TileParams<float> &, int, hipStream_t);
template hipError_t launch_tile_scatter<float>(const TileParams<float> &, hipStream_t);

}  // namespace rb
