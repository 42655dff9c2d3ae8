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
__device__ __forceinline__ int64_t rec_at(const TileParams<T> &p, int ph, int t, int f, int slot) {
    return (((int64_t)ph * p.ntile + t) * TILE_NF + f) * p.cap + slot;
}
template <typename T>
__device__ __forceinline__ int64_t bin_at(const TileParams<T> &p, int ph, int t, int slot) {
    return ((int64_t)ph * p.ntile + t) * p.cap + slot;
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
    const T f[TILE_NF] = {sn.x, sn.y, sn.z, st[l], st[p.S + l], st[2 * p.S + l], st[3 * p.S + l],
                          st[4 * p.S + l], st[5 * p.S + l], st[6 * p.S + l], st[7 * p.S + l], st[8 * p.S + l],
                          st[9 * p.S + l]};
#pragma unroll
    for (int k = 0; k < TILE_NF; ++k) p.rec[rec_at(p, 0, t, k, slot)] = f[k];
    p.id[bin_at(p, 0, t, slot)] = id;
    // no history yet: the current speed (a violated bound just shortens the
    // first block)
    const float s = (float)sqroot(f[7] * f[7] + f[8] * f[8] + f[9] * f[9]) * 1.0001f;
    p.sig[bin_at(p, 0, t, slot)] = s;
    atomicMax(&p.ctl->sig_max, __float_as_uint(s));
}

// ---- bins[phase] -> canonical state (state rows, snapshot of the final step) --
template <typename T>
__global__ __launch_bounds__(256) void tile_scatter_kernel(TileParams<T> p) {
    const int t = blockIdx.x;
    const int ph = p.ctl->phase;
    const int n = min(p.count[ph * p.ntile + t], p.cap);
    Snap<T> *out = p.snap_out[(p.c0 + p.ctl->done) & 1];
    for (int slot = threadIdx.x; slot < n; slot += 256) {
        const int32_t id = p.id[bin_at(p, ph, t, slot)];
        const int64_t l = id - p.lo;
        T f[TILE_NF];
#pragma unroll
        for (int k = 0; k < TILE_NF; ++k) f[k] = p.rec[rec_at(p, ph, t, k, slot)];
        T *st = p.st_base;
#pragma unroll
        for (int k = 0; k < 10; ++k) st[k * p.S + l] = f[3 + k];
        out[id] = Snap<T>{f[0], f[1], f[2], p.cs.bound()[id]};
    }
}

// ---- one block: K steps of one tile ---------------------------------------
template <typename T, int NT>
__global__ __launch_bounds__(NT) void tile_block_kernel(TileParams<T> p) {
    constexpr int LC = NT + NT / 2;            // LDS entries: [0, NT) stepped, [NT, LC) outer ring
    constexpr int NW = NT / 64;
    __shared__ Snap<T> s_pos[2][NT];           // positions of the stepped bodies (ping-pong by step)
    __shared__ T s_x0[3][LC];                  // block-start positions
    __shared__ float s_a1[LC];                 // speed term of the displacement bound (bound_at)
    __shared__ float s_r[LC];                  // bounding radii (rounded up)
    __shared__ int32_t s_gid[LC];
    __shared__ T s_I[3][NT];                   // principal inertia of the stepped bodies
    __shared__ T s_mr[2][NT];                  // their mass and radius (LDS, not VGPRs)
    __shared__ float s_sn[NT];                 // their top speed over the block (the next block's bound)
    __shared__ uint8_t s_t[LC];                // step at which the entry is tainted (T_NEVER: never)
    __shared__ uint16_t s_list[TILE_MAXL][NT]; // neighbour lists (entry indices, ascending global id)
    __shared__ uint8_t s_nl[NT];
    __shared__ int32_t s_misc[16];
    __shared__ T s_ring[4];                    // outer ring box x0 x1 y0 y1 (fp64 values: LDS, not VGPRs)
    __shared__ int32_t s_ctot[TILE_NCOL / 64];
    // build-time aliases: load references over the lists, the column sort over s_pos[1]
    uint32_t *s_ref = reinterpret_cast<uint32_t *>(&s_list[0][0]);
    uint32_t *s_col = reinterpret_cast<uint32_t *>(&s_pos[1][0]);
    uint16_t *s_sorted = reinterpret_cast<uint16_t *>(s_col + TILE_NCOL);
    static_assert(sizeof(s_list) >= sizeof(uint32_t) * LC, "load references alias the lists");
    static_assert(sizeof(s_pos[1]) >= sizeof(uint32_t) * TILE_NCOL + sizeof(uint16_t) * LC, "column sort aliases s_pos[1]");

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
    if (tid < 16) s_misc[tid] = (tid == 4 || tid == 6) ? INT32_MAX : (tid == 5 || tid == 7) ? INT32_MIN : 0;
    if (tid == 2) s_misc[2] = (W + M + (Sfx > Sfy ? Sfx : Sfy) > p.tile) ? ERR_TILE : 0;   // ring within the 9 bins
    if (tid == 3) s_misc[3] = k_run;           // steps valid (min over owned bodies)
    if (tid == 4) { s_ring[0] = ox0; s_ring[1] = ox1; s_ring[2] = oy0; s_ring[3] = oy1; }
    __syncthreads();

    // ---- 1. the 9 bins around the tile: stepped (band) and outer (ring) entries
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
    for (int idx = tid; idx < pre[9]; idx += NT) {
        // the last bin starting at or before idx (selects: no indexed private array)
        int b = binid[0], base = 0;
#pragma unroll
        for (int u = 1; u < 9; ++u)
            if (idx >= pre[u]) { b = binid[u]; base = pre[u]; }
        const int slot = idx - base;
        const T x = p.rec[rec_at(p, ph, b, 0, slot)], y = p.rec[rec_at(p, ph, b, 1, slot)];
        const uint32_t ref = (uint32_t)b * (uint32_t)p.cap + (uint32_t)slot;
        if (!(absval(x) < T(1e9) && absval(y) < T(1e9))) {
            atomicOr(p.err, ERR_DOMAIN);       // non-finite / runaway position (rb_grid.hpp cell_of)
            continue;
        }
        if (x >= lx0 && x < lx1 && y >= ly0 && y < ly1) {
            const int e = atomicAdd(&s_misc[0], 1);
            if (e < NT) s_ref[e] = ref;
            else s_misc[2] = ERR_TILE;
        } else if (x >= ox0 && x < ox1 && y >= oy0 && y < oy1) {
            const int o = atomicAdd(&s_misc[1], 1);
            if (o < LC - NT) s_ref[NT + o] = ref;
            else s_misc[2] = ERR_TILE;
        }
    }
    __syncthreads();
    const int nl = s_misc[0] < NT ? s_misc[0] : NT, no = s_misc[1] < LC - NT ? s_misc[1] : LC - NT;

    TSTAMP(1);
    // ---- 2. records -> registers (stepped) and LDS (every entry)
    V3<T> x{}, v{}, w{};
    Q4<T> q{};
    bool own = false;
    if (tid < nl) {
        const uint32_t ref = s_ref[tid];
        const int b = (int)(ref / (uint32_t)p.cap), slot = (int)(ref % (uint32_t)p.cap);
        T f[TILE_NF];
#pragma unroll
        for (int k = 0; k < TILE_NF; ++k) f[k] = p.rec[rec_at(p, ph, b, k, slot)];
        const int32_t gid = p.id[bin_at(p, ph, b, slot)];
        const float sg = p.sig[bin_at(p, ph, b, slot)];
        x = {f[0], f[1], f[2]};
        q = {f[3], f[4], f[5], f[6]};
        v = {f[7], f[8], f[9]};
        w = {f[10], f[11], f[12]};
        s_mr[0][tid] = p.cs.mass()[gid];
        s_I[0][tid] = p.cs.ix()[gid];
        s_I[1][tid] = p.cs.iy()[gid];
        s_I[2][tid] = p.cs.iz()[gid];
        const T rad = p.cs.sx()[gid];   // spheres only: the bound is the radius
        s_mr[1][tid] = rad;
        own = tile_x(p, x.x) == tx && tile_y(p, x.y) == ty;
        s_pos[0][tid] = Snap<T>{x.x, x.y, x.z, rad};
        s_x0[0][tid] = x.x; s_x0[1][tid] = x.y; s_x0[2][tid] = x.z;
        s_a1[tid] = speed_term(p, sg);
        s_r[tid] = (float)rad * 1.000001f;
        s_gid[tid] = gid;
        s_t[tid] = T_NEVER;
        s_sn[tid] = (float)sqroot(v.x * v.x + v.y * v.y + v.z * v.z);
        if (own) atomicAdd(&s_misc[12], 1);
    }
    if (tid < no) {
        const int e = NT + tid;
        const uint32_t ref = s_ref[e];
        const int b = (int)(ref / (uint32_t)p.cap), slot = (int)(ref % (uint32_t)p.cap);
        const int32_t g = p.id[bin_at(p, ph, b, slot)];
        const float sg = p.sig[bin_at(p, ph, b, slot)];
#pragma unroll
        for (int d = 0; d < 3; ++d) s_x0[d][e] = p.rec[rec_at(p, ph, b, d, slot)];
        s_a1[e] = speed_term(p, sg);
        s_r[e] = (float)p.cs.bound()[g] * 1.000001f;
        s_gid[e] = g;
        s_t[e] = 0;                            // outer: unknown from the start
    }
    // column grid extent: the entries' xy box, and the largest pair reach
    {
        float bx0 = 3e38f, bx1 = -3e38f, by0 = 3e38f, by1 = -3e38f, smax = 0.f;
        if (tid < nl) {
            bx0 = bx1 = (float)x.x; by0 = by1 = (float)x.y;
            smax = s_a1[tid];
        }
        if (tid < no) {
            const float ex = (float)s_x0[0][NT + tid], ey = (float)s_x0[1][NT + tid];
            bx0 = fminf(bx0, ex); bx1 = fmaxf(bx1, ex); by0 = fminf(by0, ey); by1 = fmaxf(by1, ey);
            smax = fmaxf(smax, s_a1[NT + tid]);
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            bx0 = fminf(bx0, __shfl_xor(bx0, o)); bx1 = fmaxf(bx1, __shfl_xor(bx1, o));
            by0 = fminf(by0, __shfl_xor(by0, o)); by1 = fmaxf(by1, __shfl_xor(by1, o));
            smax = fmaxf(smax, __shfl_xor(smax, o));
        }
        if (lane == 0) {
            atomicMin(&s_misc[4], f2o(bx0)); atomicMax(&s_misc[5], f2o(bx1));
            atomicMin(&s_misc[6], f2o(by0)); atomicMax(&s_misc[7], f2o(by1));
            atomicMax(&s_misc[8], f2o(smax));
        }
    }
    __syncthreads();
    if (s_misc[2]) {                           // capacity: the run falls back
        if (tid == 0) { atomicOr(&ctl->acc_err, s_misc[2]); s_misc[3] = 0; }
    }
    int my_valid = k_run;
    int disp_bad = 0;
    if (s_misc[12] > 0) {                      // (uniform) a tile with bodies to step
    TSTAMP(2);
    // ---- 3. neighbour lists: counting sort of the entries by xy column
    // columns at least as wide as the largest pair reach over the block
    const float gx0 = o2f(s_misc[4]), gy0 = o2f(s_misc[6]);
    const float gx1 = o2f(s_misc[5]), gy1 = o2f(s_misc[7]);
    const float sxy = bound_at(k_s, o2f(s_misc[8]), a2[0] > a2[1] ? a2[0] : a2[1]);
    float cs = 2.0f * (float)p.rmax * 1.000001f + 2.0f * sxy + 2.0f * S_EPS;
    int ncx = (int)((gx1 - gx0) / cs) + 1, ncy = (int)((gy1 - gy0) / cs) + 1;
    while ((int64_t)ncx * ncy > TILE_NCOL) {
        cs *= 1.25f;
        ncx = (int)((gx1 - gx0) / cs) + 1;
        ncy = (int)((gy1 - gy0) / cs) + 1;
    }
    auto col_of = [&](float ex, float ey) {
        int cx = (int)((ex - gx0) / cs), cy = (int)((ey - gy0) / cs);
        cx = cx < 0 ? 0 : cx >= ncx ? ncx - 1 : cx;
        cy = cy < 0 ? 0 : cy >= ncy ? ncy - 1 : cy;
        return cy * ncx + cx;
    };
    for (int c = tid; c < TILE_NCOL; c += NT) s_col[c] = 0;
    __syncthreads();
    int col_l = -1, col_o = -1;
    if (tid < nl) { col_l = col_of((float)x.x, (float)x.y); atomicAdd(&s_col[col_l], 1u); }
    if (tid < no) { col_o = col_of((float)s_x0[0][NT + tid], (float)s_x0[1][NT + tid]); atomicAdd(&s_col[col_o], 1u); }
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
    // now s_col[c] = end of column c = start of column c + 1
    if (tid < nl) {
        int nlist = 0;
        const int me_c = col_l, mcx = me_c % ncx, mcy = me_c / ncx;
        const float ra = s_r[tid], a1 = s_a1[tid];
        const float sa0 = bound_at(k_s, a1, a2[0]), sa1 = bound_at(k_s, a1, a2[1]), sa2 = bound_at(k_s, a1, a2[2]);
        bool over = false;
        for (int dy = -1; dy <= 1; ++dy) {
            const int yy = mcy + dy;
            if (yy < 0 || yy >= ncy) continue;
            for (int dx = -1; dx <= 1; ++dx) {
                const int xx = mcx + dx;
                if (xx < 0 || xx >= ncx) continue;
                const int c = yy * ncx + xx;
                const uint32_t c0 = c ? s_col[c - 1] : 0u, c1 = s_col[c];
                for (uint32_t u = c0; u < c1; ++u) {
                    const int mi = s_sorted[u];
                    if (mi == tid) continue;
                    const float rr = ra + s_r[mi];
                    const float b1 = s_a1[mi];
                    if (!(fabsf((float)(x.x - s_x0[0][mi])) < rr + sa0 + bound_at(k_s, b1, a2[0]) + S_EPS)) continue;
                    if (!(fabsf((float)(x.y - s_x0[1][mi])) < rr + sa1 + bound_at(k_s, b1, a2[1]) + S_EPS)) continue;
                    if (!(fabsf((float)(x.z - s_x0[2][mi])) < rr + sa2 + bound_at(k_s, b1, a2[2]) + S_EPS)) continue;
                    if (nlist == TILE_MAXL) { over = true; continue; }
                    // insert by global id (the canonical partner order)
                    const int32_t gm = s_gid[mi];
                    int k = nlist;
                    while (k > 0 && s_gid[s_list[k - 1][tid]] > gm) { s_list[k][tid] = s_list[k - 1][tid]; --k; }
                    s_list[k][tid] = (uint16_t)mi;
                    ++nlist;
                }
            }
        }
        s_nl[tid] = (uint8_t)nlist;
        if (over) s_t[tid] = 0;                // its list cannot be complete: unknown from the start
    }
    __syncthreads();

    TSTAMP(3);
    // ---- 4. K steps
    if (tid < nl && own && s_t[tid] == 0) my_valid = 0;
    for (int s = 0; s < k_run; ++s) {
        const int cur = s & 1;
        if (tid < nl && s_t[tid] > s) {
            const T m = s_mr[0][tid], rad = s_mr[1][tid];
            const int nlist = s_nl[tid];
            // a body beyond the ring (moved at most its bound) in reach?
            const T fx = (T)bound_at(s, af, a2[0]) + rad + p.rmax, fy = (T)bound_at(s, af, a2[1]) + rad + p.rmax;
            bool taint = (x.x - s_ring[0] < fx) || (s_ring[1] - x.x < fx) || (x.y - s_ring[2] < fy) ||
                         (s_ring[3] - x.y < fy);
            for (int k = 0; k < nlist && !taint; ++k) {
                const int mi = s_list[k][tid];
                if (s_t[mi] > s) continue;
                // a tainted neighbour: could its true position (within its
                // bound of step s) reach this body?
                T g2 = T(0);
                const float b1 = s_a1[mi];
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    const T xd = d == 0 ? x.x : d == 1 ? x.y : x.z;
                    T gap = absval(xd - s_x0[d][mi]) - (T)bound_at(s, b1, a2[d]);
                    gap = gap > T(0) ? gap : T(0);
                    g2 += gap * gap;
                }
                const T rr = rad + (T)s_r[mi] + T(S_EPS);
                taint = g2 < rr * rr;
            }
            if (taint) {
                s_t[tid] = (uint8_t)(s + 1);
                if (own && my_valid > s) my_valid = s;
            } else {
                // one reference step (rb_kernels.hip body_update, same operation order)
                InvI<T> inv{&s_I[0][tid], NT, q, false, {}};
                {
                    const V3<T> F = {m * p.g[0], m * p.g[1], m * p.g[2]};      // collision.py:66-69
                    v = {v.x + (F.x / m) * p.dt, v.y + (F.y / m) * p.dt, v.z + (F.z / m) * p.dt};
                }
                const T kk = impulse_k(m);
                // plane contacts (plane order), then partners in ascending id:
                // one solve site for both (fewer inlined copies, fewer live registers)
                const int npl = p.n_planes, ktot = npl + nlist;
                for (int k = 0; k < ktot; ++k) {
                    Contact<T> con;
                    V3<T> n;
                    if (k < npl) {
                        const V3<T> pn = {p.pn[k][0], p.pn[k][1], p.pn[k][2]};
                        const V3<T> pp = {p.pp[k][0], p.pp[k][1], p.pp[k][2]};
                        if (!plane_sphere(pn, pp, x, rad, con)) continue;
                        n = con.frame;
                    } else {
                        const int mi = s_list[k - npl][tid];
                        if (s_t[mi] <= s) continue;    // tainted and out of reach (tested above)
                        const Snap<T> pe = s_pos[cur][mi];
                        const V3<T> cj = {pe.x, pe.y, pe.z};
                        if (!sphere_sphere_hit(x, rad, cj, pe.r)) continue;
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
        // wave offsets in wave order (deterministic slots)
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
        const T f[TILE_NF] = {x.x, x.y, x.z, q.w, q.x, q.y, q.z, v.x, v.y, v.z, w.x, w.y, w.z};
#pragma unroll
        for (int k = 0; k < TILE_NF; ++k) p.rec[rec_at(p, 1 - ph, (int)t, k, slot)] = f[k];
        p.id[bin_at(p, 1 - ph, (int)t, slot)] = s_gid[tid];
        p.sig[bin_at(p, 1 - ph, (int)t, slot)] = s_sn[tid] * 1.0001f;
    }
    __syncthreads();

    TSTAMP(5);
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
                const int kn = k_run < k_s ? k_run : (k_s < p.kmax ? k_s + 1 : p.kmax);
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
    if (nt == 512) hipLaunchKernelGGL((tile_block_kernel<T, 512>), dim3((unsigned)p.ntile), dim3(512), 0, s, p);
    else if (nt == 768) hipLaunchKernelGGL((tile_block_kernel<T, 768>), dim3((unsigned)p.ntile), dim3(768), 0, s, p);
    else return hipErrorInvalidValue;
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
