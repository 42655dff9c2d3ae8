// rb_tiles.hip — the cell-ordered tile form of the step (rb_internal.hpp
// TileParams): sphere worlds on one rank.
//
// One launch per reference step, one workgroup per tile slot.  The step is
// the reference's: contacts from the step-start positions of every body
// (mj_forward, collision.py:57 / multi_sphere_bounce.py:43), then per body
// gravity, its plane contacts and its sphere partners in ascending id, each
// through compute_collision_impulse_friction (collision.py:7-48) and
// apply_impulse_friction (physics_utils.py:25-49), then the integration
// (collision.py:90-100) — Jacobi across bodies, Gauss-Seidel within one
// (collision.py:72-88).  The per-body arithmetic is rb_body.hpp's, shared
// with the hashed-cell kernels, so both forms step a body bit-identically;
// what differs is how a body finds its partners:
//
//   hashed cells (rb_kernels.hip): each body reads 8 bucket heads, then
//     its candidates' snapshots — two dependent rounds of random gathers per
//     lane — and claims a slot in the next table with two atomics;
//   tiles (here): a workgroup reads the column tables of its 3 x 3 bins, then
//     every record of its window of columns with coalesced loads (one thread
//     per window column), placed in LDS sorted by column (the counts are
//     known from the tables before a record arrives); each body searches its
//     2 x 2 nearest columns — two runs of the window — in LDS.  The next bin
//     is written sorted by column from an LDS counting sort.
//
// Launch shape: 128 threads (two waves) per slot; a slot steps at most 128
// bodies (more raises ERR_TILE: the host replays the run with the hashed
// forms).  The kernel is instantiated per tile width (tc = 4..8 columns), so
// every column index is arithmetic on constants.  Slots are dealt so that
// each XCD steps one contiguous band of slot rows (a bin is read by the
// workgroups of its neighbours, mostly on the same L2).
#include "rb_device.hpp"
#include "rb_grid.hpp"
#include "rb_internal.hpp"
#include "rb_body.hpp"

// diagnostic build only (RB_TILE_STAMPS=1, scripts/tile_stamps.py): per-
// workgroup s_memtime stamps at the phase ends, and s_memrealtime (100 MHz,
// comparable across XCDs) at the start and the end
#ifndef RB_TILE_STAMPS
#define RB_TILE_STAMPS 0
#endif
#if RB_TILE_STAMPS
__device__ unsigned long long rb_tile_stamp_buf[1 << 14][12];
#define TSTAMP(k)                                                                                  \
    do {                                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                                         \
        unsigned long long t_;                                                                     \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                 \
        __builtin_amdgcn_sched_barrier(0);                                                         \
        if (threadIdx.x == 0 && blockIdx.x < (1u << 14)) rb_tile_stamp_buf[blockIdx.x][k] = t_;    \
        if (k == 0 || k == 9) {                                                                    \
            unsigned long long r_;                                                                 \
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r_)::"memory");         \
            if (threadIdx.x == 0 && blockIdx.x < (1u << 14)) rb_tile_stamp_buf[blockIdx.x][k == 0 ? 10 : 11] = r_; \
        }                                                                                          \
    } while (0)
#else
#define TSTAMP(k) do {} while (0)
#endif

namespace rb {

static_assert((TILE_TC_MAX + 2) * (TILE_TC_MAX + 2) + 1 <= TILE_OFFW &&
              (TILE_TC_MAX + 2) * (TILE_TC_MAX + 2) <= TILE_THREADS, "column tables");
static_assert(TILE_WMAX + TILE_FARWIN <= 65536, "window indices are 16-bit");

__device__ __forceinline__ int32_t pmod(int32_t a, int32_t m) {
    const int32_t r = a % m;
    return r < 0 ? r + m : r;
}
__device__ __forceinline__ int32_t fdiv(int32_t a, int32_t b) {   // floor(a / b), b > 0
    const int32_t q = a / b;
    return (a % b < 0) ? q - 1 : q;
}
// column of a coordinate and the position inside it (false: non-finite or
// out of range, as cell_of)
template <typename T> __device__ __forceinline__ bool col_of(T x, T inv, int32_t &c, T &frac) {
    const T f = x * inv;
    if (!(absval(f) < T(1 << 29))) return false;
    const T fl = (T)__builtin_floor((double)f);
    c = (int32_t)fl;
    frac = f - fl;
    return true;
}

// The bins a window column's records come from: along each axis the slot's
// own bin, and for the two outer columns of each side the neighbour's (at
// most one neighbour per axis).  Pair a (< n), in the order y outer, x
// inner: bin j = (dy + 1) * 3 + (dx + 1) and that bin's own column index.
// Columns are numbered row-major over the extended tile (-1 .. tc)^2.
struct ColSrc {
    int n;
    int j[4], c[4];
};
template <int TC> __device__ __forceinline__ ColSrc col_sources(int vx, int vy) {
    constexpr int EXT = TC + 2;
    int xd1 = 0, xb1 = vx, nx = 1;
    if (vx >= TC - 1) { xd1 = 1; xb1 = vx - TC; nx = 2; }
    else if (vx <= 0) { xd1 = -1; xb1 = vx + TC; nx = 2; }
    int yd1 = 0, yb1 = vy, ny = 1;
    if (vy >= TC - 1) { yd1 = 1; yb1 = vy - TC; ny = 2; }
    else if (vy <= 0) { yd1 = -1; yb1 = vy + TC; ny = 2; }
    ColSrc s;
    s.n = nx * ny;
    const int xdb = nx == 2 ? xd1 : 0, xbb = nx == 2 ? xb1 : vx;   // pair 1: x-neighbour, or y-neighbour
    const int ydb = nx == 2 ? 0 : yd1, ybb = nx == 2 ? vy : yb1;
    s.j[0] = 4;                              s.c[0] = (vy + 1) * EXT + (vx + 1);
    s.j[1] = (ydb + 1) * 3 + (xdb + 1);      s.c[1] = (ybb + 1) * EXT + (xbb + 1);
    s.j[2] = (yd1 + 1) * 3 + 1;              s.c[2] = (yb1 + 1) * EXT + (vx + 1);
    s.j[3] = (yd1 + 1) * 3 + (xd1 + 1);      s.c[3] = (yb1 + 1) * EXT + (xb1 + 1);
    return s;
}

// inclusive scan over the wave's 64 lanes with DPP (register-to-register,
// no LDS round trips): row_shr 1, 2, 4, 8 inside each row of 16 lanes, then
// row_bcast:15 and row_bcast:31 carry the rows' totals upward
__device__ __forceinline__ int wave_scan_incl(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);   // row_bcast:15 into rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);   // row_bcast:31 into rows 2, 3
    return x;
}
// exclusive scan of one value per thread over the workgroup (128 threads);
// s_tmp[2] is free again after the next barrier
__device__ __forceinline__ int block_scan_excl(int v, int32_t *s_tmp, int &total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int x = wave_scan_incl(v);
    if (lane == 63) s_tmp[wv] = x;
    __syncthreads();
    const int w0 = s_tmp[0];
    total = w0 + s_tmp[1];
    return x - v + (wv ? w0 : 0);
}

template <typename T>
__device__ __forceinline__ void tile_fail(const TileParams<T> &p, int why) {
    atomicOr(p.why, why);
    atomicOr(p.sp.err, ERR_TILE);
}

// OCC: waves per SIMD the registers are sized for — 2 (fp64 192 VGPRs), or 3
// (168, no scratch at MAXP 16) for grids of more slots than fit the GPU at
// once at 2, where throughput, not one workgroup's chain, sets the step time
// (4M flat spheres 600 -> 540 us; C3's 900 slots 16.2 -> 17.4 us, so not there)
template <typename T, int MAXP, int TC, int OCC>
__global__ __launch_bounds__(TILE_THREADS) __attribute__((amdgpu_waves_per_eu(OCC, OCC)))
void tile_step_kernel(const int32_t *cur_off, int32_t ntx, int32_t nty, const uint32_t *gen_cur, const int32_t *err,
                      const unsigned long long *far_hdr, TileParams<T> p) {
    constexpr int EXT = TC + 2, NCOL = EXT * EXT, NQ = (NCOL + 1 + 3) / 4;
    // window records: [0, W) the bins', far bodies from FBASE, then one
    // dummy slot (stores past a column's records)
    constexpr int FBASE = TILE_WMAX, WCAP = FBASE + TILE_FARWIN;
    __shared__ __attribute__((aligned(16))) int32_t s_off[9][NQ * 4];
    __shared__ int32_t s_vstart[NCOL + 1];          // window column starts (row-major, extended tile)
    // window positions: fp64 in two planes (x, y | z, r), fp32 one (x, y, z, r)
    __shared__ __attribute__((aligned(16))) T s_pw[4 * (WCAP + 1)];
    auto wpos = [&](int f) -> Snap<T> {
        if constexpr (sizeof(T) == 8) return Snap<T>{s_pw[2 * f], s_pw[2 * f + 1], s_pw[2 * (WCAP + 1) + 2 * f], s_pw[2 * (WCAP + 1) + 2 * f + 1]};
        else return Snap<T>{s_pw[4 * f], s_pw[4 * f + 1], s_pw[4 * f + 2], s_pw[4 * f + 3]};
    };
    auto set_wpos = [&](int f, const Snap<T> &v) {
        if constexpr (sizeof(T) == 8) {
            s_pw[2 * f] = v.x; s_pw[2 * f + 1] = v.y;
            s_pw[2 * (WCAP + 1) + 2 * f] = v.z; s_pw[2 * (WCAP + 1) + 2 * f + 1] = v.r;
        } else {
            s_pw[4 * f] = v.x; s_pw[4 * f + 1] = v.y; s_pw[4 * f + 2] = v.z; s_pw[4 * f + 3] = v.r;
        }
    };
    __shared__ __attribute__((aligned(16))) int32_t s_id[WCAP + 1];   // id words
    __shared__ T s_fst[TILE_FARWIN][TILE_STW];      // own far bodies' state (staged by the far scan)
    __shared__ uint16_t s_pl[MAXP][TILE_THREADS];   // partners in discovery order (window index)
    __shared__ int32_t s_ocnt[NCOL];
    __shared__ int32_t s_ostart[NCOL + 1];
    __shared__ uint16_t s_fown[TILE_FARWIN];
    __shared__ int32_t s_misc[8];                   // 0 far in window, 1 far owned, 2-3 scan, 4 error, 5 piles
    __shared__ int32_t s_slot[9];

    const int tid = threadIdx.x;
    TSTAMP(0);
    const int nslots = (int)gridDim.x;
    // XCD-aware: blocks b and b + 8 share an XCD; give each XCD a contiguous
    // band of slots
    const int b = (int)blockIdx.x, xq = nslots / (int)N_XCD, xr = nslots % (int)N_XCD, xx = b % (int)N_XCD;
    const int slot = xx * xq + (xx < xr ? xx : xr) + b / (int)N_XCD;
    const int sx = slot % ntx, sy = slot / ntx;
    const uint32_t gen = *gen_cur;
    const int32_t err0 = *err;
    const unsigned long long fh = *far_hdr;

    // ---- 1. the 3 x 3 bins' column tables (one round trip) -----------------
    for (int k = tid; k < 9 * NQ; k += TILE_THREADS) {
        const int j = k / NQ, qd = k - j * NQ;
        const int bx = pmod(sx + j % 3 - 1, ntx), by = pmod(sy + j / 3 - 1, nty);
        const int4 v = reinterpret_cast<const int4 *>(cur_off + (int64_t)(by * ntx + bx) * TILE_OFFW)[qd];
        reinterpret_cast<int4 *>(&s_off[j][0])[qd] = v;
    }
    if (tid < 9) s_slot[tid] = pmod(sy + tid / 3 - 1, nty) * ntx + pmod(sx + tid % 3 - 1, ntx);
    if (tid < 8) s_misc[tid] = 0;
    if (tid < NCOL) s_ocnt[tid] = 0;
    if (err0 & ERR_TILE) return;                     // the run already failed: it is replayed anyway
    __syncthreads();
    TSTAMP(1);

    // ---- 2. the window's column starts, before any record ------------------
    constexpr int WR = 6;                            // records per column staged in registers
    int cnt = 0;
    ColSrc cs{};
    int64_t src_base[4] = {0, 0, 0, 0};
    int src_n[4] = {0, 0, 0, 0};
    if (tid < NCOL) {
        cs = col_sources<TC>(tid % EXT - 1, tid / EXT - 1);
        bool bad = false;
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            if (a >= cs.n) break;
            const int lo = s_off[cs.j[a]][cs.c[a]], hi = s_off[cs.j[a]][cs.c[a] + 1];
            bad |= !(lo >= 0 && lo <= hi && hi <= p.cap);
            src_base[a] = (int64_t)s_slot[cs.j[a]] * p.cap + lo;
            src_n[a] = hi - lo;
            cnt += hi - lo;
        }
        if (bad) { s_misc[4] = 1; cnt = 0; }
        if (cnt > WR) s_misc[5] = 1;                // a pile: loaded after the first WR (below)
    }
    int W;
    const int ex = block_scan_excl(cnt, &s_misc[2], W);
    if (tid < NCOL) s_vstart[tid] = ex;
    if (tid == 0) s_vstart[NCOL] = W;
    const int32_t nfar = (uint32_t)(fh >> 32) == gen ? (int32_t)(uint32_t)fh : 0;
    if (s_misc[4] || W > TILE_WMAX || nfar > TILE_FARMAX) {
        if (tid == 0) tile_fail(p, s_misc[4] ? TILE_WHY_CAP : W > TILE_WMAX ? TILE_WHY_WINDOW : TILE_WHY_FAR);
        return;
    }
    __syncthreads();
    TSTAMP(2);

    // ---- 3. the records: own bodies' first (their loads are the oldest, so a
    // body's arithmetic waits for them only), then each window column's
    // (thread k, column k) into registers; those land in LDS after the own
    // bodies' gravity, plane contacts and inv(I_w), which run meanwhile
    // own bodies: the interior rows' runs of the window, row by row
    int n_own = 0, widx = 0, row = 0;
#pragma unroll
    for (int r = 0; r < TC; ++r) {
        const int a = s_vstart[(r + 1) * EXT + 1], e = s_vstart[(r + 1) * EXT + TC + 1];
        if (tid >= n_own && tid < n_own + (e - a)) { widx = a + tid - n_own; row = r; }
        n_own += e - a;
    }
    const bool own_bin = tid < n_own;
    // (the index under the branch, the loads outside it — lanes past the own
    // bodies fetch record 0 — so that the wait before the arithmetic counts
    // them exactly, and the window's loads below issue behind them unwaited)
    int64_t g = 0;
    if (own_bin) {
        int k = (row + 1) * EXT + 1;
#pragma unroll
        for (int c = 1; c < TC; ++c)
            if (s_vstart[(row + 1) * EXT + 1 + c] <= widx) k = (row + 1) * EXT + 1 + c;
        const ColSrc ks = col_sources<TC>(k % EXT - 1, k / EXT - 1);
        int r = widx - s_vstart[k];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            if (a >= ks.n) break;
            const int lo = s_off[ks.j[a]][ks.c[a]], n = s_off[ks.j[a]][ks.c[a] + 1] - lo;
            if (r >= 0 && r < n) g = (int64_t)s_slot[ks.j[a]] * p.cap + lo + r;
            r -= n;
        }
    }
    Snap<T> self = p.cur.pos[g];
    int32_t idw = p.cur.id[g];
    const T *stp = p.cur.st + g * TILE_STW;
    Q4<T> q = {stp[0], stp[1], stp[2], stp[3]};
    V3<T> v = {stp[4], stp[5], stp[6]}, w = {stp[7], stp[8], stp[9]};
    // the window: up to WR records per column in registers (the rest, a pile,
    // after); slots past the column's count load record 0 (one shared address)
    // (every lane issues them — lanes past the window's columns fetch record
    // 0 — so no branch hides their count from the wait before the arithmetic)
    Snap<T> rsn[WR];
    int32_t rid[WR];
    {
#pragma unroll
        for (int u = 0; u < WR; ++u) {
            int rr = u;
            int64_t g = 0;
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                if (rr >= 0 && rr < src_n[a]) g = src_base[a] + rr;
                rr -= src_n[a];
            }
            rsn[u] = p.cur.pos[g];
            rid[u] = p.cur.id[g];
        }
    }

    // ---- 4. one lane per own body ------------------------------------------
    // a4 gravity, K2 plane contacts (the first in a body's contact order) and
    // inv(I_w), eagerly (rb_body.hpp; value-identical to evaluating it at the
    // first impulse)
    const StepParams<T> &sp = p.sp;
    LazyInvI<T> invI;
    T m = 0, kimp = 0;
    int32_t nrec = 0;
    V3<T> x{};
    auto phys_a = [&]() {
        x = {self.x, self.y, self.z};
        V3<T> I;
        if (p.ntypes == 1) {
            // one type (every body alike): the kernel's arguments, no memory
            // access (a load here would wait for every window load before it)
            m = p.types[0][0];
            I = {p.types[0][1], p.types[0][2], p.types[0][3]};
        } else {
            // a few types: selected by value (the arguments read first, so the
            // select is not turned into a selected address and a load)
            const int ty = (int)((uint32_t)idw >> TILE_ID_BITS);
            T tv[TILE_TYPES][4];
#pragma unroll
            for (int t = 0; t < TILE_TYPES; ++t)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    tv[t][c] = p.types[t][c];
                    asm volatile("" : "+s"(tv[t][c]));
                }
            m = tv[0][0];
            I = {tv[0][1], tv[0][2], tv[0][3]};
#pragma unroll
            for (int t = 1; t < TILE_TYPES; ++t)
                if (ty == t) { m = tv[t][0]; I = {tv[t][1], tv[t][2], tv[t][3]}; }
        }
        invI.I = I;
        invI.q = q;
        invI.get();
        const int32_t id = idw & TILE_ID_MASK;
        apply_force<T, false>(sp, id, m, invI, v, w);   // (no xfrc: tile_eligible)
        kimp = impulse_k(m);
        for (int pl = 0; pl < sp.n_planes; ++pl) {
            const V3<T> pn = {sp.pn[pl][0], sp.pn[pl][1], sp.pn[pl][2]};
            const V3<T> pp = {sp.pp[pl][0], sp.pp[pl][1], sp.pp[pl][2]};
            Contact<T> con;
            if (!plane_sphere(pn, pp, x, self.r, con)) continue;
            record(sp, id, nrec, -1 - pl, 0, con.dist);
            solve_contact(sp, con, x, con.frame, m, kimp, invI, v, w);
        }
    };
    if (own_bin) phys_a();
    TSTAMP(3);
    if (tid < NCOL) {
#pragma unroll
        for (int u = 0; u < WR; ++u) {
            const int f = u < cnt ? ex + u : WCAP;   // (past the column's records: the dummy slot)
            set_wpos(f, rsn[u]);
            s_id[f] = rid[u];
        }
    }
    // piles: the records past WR of every column, spread over all lanes (one
    // round trip for most piles); a window index's column by binary search of
    // the starts (the last start <= it is the non-empty column holding it)
    if (s_misc[5]) {
        for (int i = tid; i < W; i += TILE_THREADS) {
            int lo = 0, hi = NCOL;
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (s_vstart[mid] <= i) lo = mid; else hi = mid;
            }
            int rr = i - s_vstart[lo];
            if (rr < WR) continue;
            const ColSrc ks = col_sources<TC>(lo % EXT - 1, lo / EXT - 1);
            int64_t g = 0;
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                if (a >= ks.n) break;
                const int o = s_off[ks.j[a]][ks.c[a]], n = s_off[ks.j[a]][ks.c[a] + 1] - o;
                if (rr >= 0 && rr < n) g = (int64_t)s_slot[ks.j[a]] * p.cap + o + rr;
                rr -= n;
            }
            set_wpos(i, p.cur.pos[g]);
            s_id[i] = p.cur.id[g];
        }
    }

    // far bodies inside the window (the far list: rare)
    const int Px = ntx * TC, Py = nty * TC;
    for (int i = tid; i < nfar; i += TILE_THREADS) {
        const Snap<T> sn = p.cur.far_pos[i];
        int32_t cx, cy;
        T fr;
        col_of(sn.x, p.inv_col, cx, fr);             // (checked when the body was listed)
        col_of(sn.y, p.inv_col, cy, fr);
        const int vx = pmod(cx - sx * TC + 1, Px) - 1, vy = pmod(cy - sy * TC + 1, Py) - 1;
        if (vx > TC || vy > TC) continue;
        const int qf = atomicAdd(&s_misc[0], 1);
        if (qf >= TILE_FARWIN) { s_misc[4] = 1; continue; }
        const int f = FBASE + qf;
        set_wpos(f, sn);
        s_id[f] = p.cur.far_id[i];
        if (vx >= 0 && vx < TC && vy >= 0 && vy < TC) {
            const int o = atomicAdd(&s_misc[1], 1);
            s_fown[o] = (uint16_t)f;
            const T *stp = p.cur.far_st + (int64_t)i * TILE_STW;
#pragma unroll
            for (int d = 0; d < TILE_STW; ++d) s_fst[o][d] = stp[d];
        }
    }
    __syncthreads();
    const int nfw = s_misc[0] < TILE_FARWIN ? s_misc[0] : TILE_FARWIN;
    const int n_tot = n_own + s_misc[1];
    if (s_misc[4] || n_tot > TILE_THREADS) {
        if (tid == 0) tile_fail(p, s_misc[4] ? TILE_WHY_WINDOW : TILE_WHY_CAP);
        return;
    }
    const bool act = tid < n_tot;
    if (act && !own_bin) {                           // a far body of this slot (state staged in LDS)
        widx = s_fown[tid - n_own];
        self = wpos(widx);
        idw = s_id[widx];
        const T *o = s_fst[tid - n_own];
        q = {o[0], o[1], o[2], o[3]};
        v = {o[4], o[5], o[6]};
        w = {o[7], o[8], o[9]};
        phys_a();
    }
    const int32_t id = idw & TILE_ID_MASK;
    int ex_ = 0, ey_ = 0, rank = 0;
    bool far = false, placed = false;
    Q4<T> qn{};
    if (act) {
        // K1: the 2 x 2 nearest columns, two runs of two columns each
        int32_t cx = 0, cy = 0;
        T frx = 0, fry = 0;
        col_of(self.x, p.inv_col, cx, frx);
        col_of(self.y, p.inv_col, cy, fry);
        const int vx = cx - fdiv(cx, TC) * TC, vy = cy - fdiv(cy, TC) * TC;
        const int c0 = frx >= T(0.5) ? vx : vx - 1;
        const int r1 = fry >= T(0.5) ? vy + 1 : vy - 1;
        const int k1 = (vy + 1) * EXT + c0 + 1, k2 = (r1 + 1) * EXT + c0 + 1;
        const int a1 = s_vstart[k1], n1 = s_vstart[k1 + 2] - a1;
        const int a2 = s_vstart[k2], n2 = s_vstart[k2 + 2] - a2;
        const int ncand = n1 + n2;
        int np_ = 0;
        for (int i0 = 0; i0 < ncand; i0 += 4) {
            int fu[4];
            Snap<T> cu[4];
            int32_t iu[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = i0 + u;
                fu[u] = i < n1 ? a1 + i : a2 + (i - n1);
                cu[u] = wpos(fu[u]);
                iu[u] = s_id[fu[u]] & TILE_ID_MASK;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (i0 + u >= ncand || iu[u] == id) continue;
                if (sphere_sphere_hit(x, self.r, V3<T>{cu[u].x, cu[u].y, cu[u].z}, cu[u].r)) {
                    if (np_ < MAXP) s_pl[np_][tid] = (uint16_t)fu[u];
                    ++np_;
                }
            }
        }
        for (int f = FBASE; f < FBASE + nfw; ++f) {
            const Snap<T> c = wpos(f);
            if ((s_id[f] & TILE_ID_MASK) == id) continue;
            if (sphere_sphere_hit(x, self.r, V3<T>{c.x, c.y, c.z}, c.r)) {
                if (np_ < MAXP) s_pl[np_][tid] = (uint16_t)f;
                ++np_;
            }
        }
        TSTAMP(4);
        if (np_ > MAXP) {
            tile_fail(p, TILE_WHY_PARTNERS);
            np_ = MAXP;
        }
        TSTAMP(5);
        // K2: the partners in the canonical order, ascending id (collision.py:72-88
        // walks MuJoCo's contact list; SURVEY §7 hard part 1), each selected as
        // the next larger id — no sorted copy in LDS, which leaves room for a
        // sixth workgroup per CU
        int32_t prev = -1;
        for (int a = 0; a < np_; ++a) {
            int f = 0;
            int32_t j = INT32_MAX;
            for (int c = 0; c < np_; ++c) {
                const int fc = s_pl[c][tid];
                const int32_t ic = s_id[fc] & TILE_ID_MASK;
                if (ic > prev && ic < j) {
                    j = ic;
                    f = fc;
                }
            }
            prev = j;
            const Snap<T> c = wpos(f);
            const V3<T> cj = {c.x, c.y, c.z};
            Contact<T> con;
            V3<T> n;
            if (id < j) {                                // this body is geom1
                sphere_sphere(x, self.r, cj, c.r, con);
                n = sp.oriented ? V3<T>{-con.frame.x, -con.frame.y, -con.frame.z} : con.frame;
            } else {
                sphere_sphere(cj, c.r, x, self.r, con);
                n = con.frame;
            }
            record(sp, id, nrec, j, 16, con.dist);
            solve_contact(sp, con, x, n, m, kimp, invI, v, w);
        }
        if (sp.rec_count) sp.rec_count[id] = nrec;
        TSTAMP(6);
        integrate_pose(x, qn, q, v, w, sp.dt);

        // the body's column after the step, relative to its tile at the start
        int32_t cx2, cy2;
        T fr;
        if (!col_of(x.x, p.inv_col, cx2, fr) || !col_of(x.y, p.inv_col, cy2, fr)) {
            tile_fail(p, TILE_WHY_DOMAIN);
        } else {
            ex_ = cx2 - (cx - vx);
            ey_ = cy2 - (cy - vy);
            far = ex_ < -1 || ex_ > TC || ey_ < -1 || ey_ > TC;
            placed = !far;
            if (placed) rank = atomicAdd(&s_ocnt[(ey_ + 1) * EXT + ex_ + 1], 1);
        }
    }
    __syncthreads();
    TSTAMP(7);

    // ---- 5. the next bin, sorted by column; far bodies to the far list -----
    int n_out;
    const int oex = block_scan_excl(tid < NCOL ? s_ocnt[tid] : 0, &s_misc[2], n_out);
    if (tid < NCOL) s_ostart[tid] = oex;
    if (n_out > p.cap) {
        if (tid == 0) tile_fail(p, TILE_WHY_CAP);
        return;
    }
    int32_t *noff = p.next.off + (int64_t)slot * TILE_OFFW;
    if (tid < NCOL) noff[tid] = oex;
    if (tid == 0) noff[NCOL] = n_out;
    __syncthreads();
    TSTAMP(8);
    if (placed) {
        const int64_t g = (int64_t)slot * p.cap + s_ostart[(ey_ + 1) * EXT + ex_ + 1] + rank;
        p.next.pos[g] = Snap<T>{x.x, x.y, x.z, self.r};
        p.next.id[g] = idw;
        T *o = p.next.st + g * TILE_STW;
        o[0] = qn.w; o[1] = qn.x; o[2] = qn.y; o[3] = qn.z;
        o[4] = v.x; o[5] = v.y; o[6] = v.z;
        o[7] = w.x; o[8] = w.y; o[9] = w.z;
    } else if (far) {
        atomicMax(p.next.far_hdr, (unsigned long long)(gen + 1u) << 32);
        const uint32_t fi = (uint32_t)atomicAdd(p.next.far_hdr, 1ull);
        if (fi >= (uint32_t)TILE_FARMAX) {
            tile_fail(p, TILE_WHY_FAR);
        } else {
            p.next.far_pos[fi] = Snap<T>{x.x, x.y, x.z, self.r};
            p.next.far_id[fi] = idw;
            T *o = p.next.far_st + (int64_t)fi * TILE_STW;
            o[0] = qn.w; o[1] = qn.x; o[2] = qn.y; o[3] = qn.z;
            o[4] = v.x; o[5] = v.y; o[6] = v.z;
            o[7] = w.x; o[8] = w.y; o[9] = w.z;
        }
    }
    if (b == 0 && tid == 0) *p.gen_next = gen + 1u;
    TSTAMP(9);
}

// ---- bins <-> the id-ordered state -----------------------------------------
template <typename T>
__device__ __forceinline__ bool tile_place(const TileIO<T> &p, const Snap<T> &sn, int64_t &slot, int &e) {
    int32_t cx, cy;
    T fr;
    if (!col_of(sn.x, p.inv_col, cx, fr) || !col_of(sn.y, p.inv_col, cy, fr)) return false;
    const int32_t tx = fdiv(cx, p.tc), ty = fdiv(cy, p.tc);
    slot = (int64_t)pmod(ty, p.nty) * p.ntx + pmod(tx, p.ntx);
    e = (cy - ty * p.tc + 1) * (p.tc + 2) + (cx - tx * p.tc + 1);
    return true;
}

template <typename T>
__global__ __launch_bounds__(256) void tile_count_kernel(TileIO<T> p) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= p.n) return;
    int64_t slot;
    int e;
    if (!tile_place(p, p.snap[b], slot, e)) {
        atomicOr(p.why, TILE_WHY_DOMAIN);
        atomicOr(p.err, ERR_TILE);
        return;
    }
    atomicAdd(p.bins.off + slot * TILE_OFFW + e, 1);
}

template <typename T>
__global__ __launch_bounds__(TILE_THREADS) void tile_scan_kernel(TileIO<T> p) {
    __shared__ int32_t s_tmp[2];
    const int ncol = (p.tc + 2) * (p.tc + 2);
    int32_t *off = p.bins.off + (int64_t)blockIdx.x * TILE_OFFW;
    const int v = threadIdx.x < ncol ? off[threadIdx.x] : 0;
    int total;
    const int ex = block_scan_excl(v, s_tmp, total);
    if (threadIdx.x < ncol) off[threadIdx.x] = ex;
    if (threadIdx.x == 0) {
        off[ncol] = total;
        if (total > p.cap) { atomicOr(p.why, TILE_WHY_CAP); atomicOr(p.err, ERR_TILE); }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void tile_scatter_kernel(TileIO<T> p) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= p.n) return;
    const Snap<T> sn = p.snap[b];
    int64_t slot;
    int e;
    if (!tile_place(p, sn, slot, e)) return;
    const int32_t k = atomicAdd(p.fill + slot * TILE_OFFW + e, 1);
    const int32_t *off = p.bins.off + slot * TILE_OFFW;
    const int32_t r = off[e] + k;
    if (r >= p.cap) return;                          // (the scan raised TILE_WHY_CAP)
    const int64_t g = slot * p.cap + r;
    p.bins.pos[g] = sn;
    p.bins.id[g] = (int32_t)b | (p.type_of ? (int32_t)p.type_of[b] << TILE_ID_BITS : 0);
    T *o = p.bins.st + g * TILE_STW;
#pragma unroll
    for (int d = 0; d < TILE_STW; ++d) o[d] = p.st.row(d)[b];
}

// The bins (and far list) of the run's last step back into the id-ordered
// state rows and snapshot — only when no step of the run raised ERR_TILE:
// then the id-ordered state still holds the start of the first failed run,
// which the host replays.  Counts the runs committed.
template <typename T>
__global__ __launch_bounds__(256) void tile_unbin_kernel(TileIO<T> p) {
    if (*p.err & ERR_TILE) return;
    const int ncol = (p.tc + 2) * (p.tc + 2);
    const int64_t slots = (int64_t)p.ntx * p.nty, total = slots * p.cap;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < total; g += stride) {
        const int64_t s = g / p.cap;
        const int32_t k = (int32_t)(g - s * p.cap);
        if (k >= p.bins.off[s * TILE_OFFW + ncol]) continue;
        const int32_t id = p.bins.id[g] & TILE_ID_MASK;
        p.snap[id] = p.bins.pos[g];
        const T *o = p.bins.st + g * TILE_STW;
#pragma unroll
        for (int d = 0; d < TILE_STW; ++d) p.st.row(d)[id] = o[d];
    }
    const unsigned long long fh = *p.bins.far_hdr;
    const int32_t nfar = (uint32_t)(fh >> 32) == *p.gen ? (int32_t)(uint32_t)fh : 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nfar && i < TILE_FARMAX; i += stride) {
        const int32_t id = p.bins.far_id[i] & TILE_ID_MASK;
        p.snap[id] = p.bins.far_pos[i];
        const T *o = p.bins.far_st + i * TILE_STW;
#pragma unroll
        for (int d = 0; d < TILE_STW; ++d) p.st.row(d)[id] = o[d];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *p.commits += 1;
}

// ---- launchers ----------------------------------------------------------------
// the fields the step's first loads need, as leading scalar arguments that
// gfx950 preloads into SGPRs (the unit is built with
// -amdgpu-kernarg-preload-count, as the step kernels' Lead in rb_kernels.hip)
#define TILE_LEAD(p) (p).cur.off, (p).ntx, (p).nty, (p).gen_cur, (p).sp.err, (p).cur.far_hdr
template <typename T, int MAXP, int OCC>
hipError_t launch_tile_step_tc(const TileParams<T> &p, hipStream_t s) {
    const dim3 grid((unsigned)(p.ntx * p.nty)), block(TILE_THREADS);
    switch (p.tc) {
    case 4: hipLaunchKernelGGL((tile_step_kernel<T, MAXP, 4, OCC>), grid, block, 0, s, TILE_LEAD(p), p); break;
    case 5: hipLaunchKernelGGL((tile_step_kernel<T, MAXP, 5, OCC>), grid, block, 0, s, TILE_LEAD(p), p); break;
    case 6: hipLaunchKernelGGL((tile_step_kernel<T, MAXP, 6, OCC>), grid, block, 0, s, TILE_LEAD(p), p); break;
    case 7: hipLaunchKernelGGL((tile_step_kernel<T, MAXP, 7, OCC>), grid, block, 0, s, TILE_LEAD(p), p); break;
    case 8: hipLaunchKernelGGL((tile_step_kernel<T, MAXP, 8, OCC>), grid, block, 0, s, TILE_LEAD(p), p); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
template <typename T> hipError_t launch_tile_step(const TileParams<T> &p, int maxp, hipStream_t s) {
    if (p.tc < TILE_TC_MIN || p.tc > TILE_TC_MAX || p.ntx < 3 || p.nty < 3 || p.cap <= 0 || p.cap > TILE_THREADS ||
        p.ntypes < 1 || p.ntypes > TILE_TYPES)
        return hipErrorInvalidValue;
    if (maxp > 16) return launch_tile_step_tc<T, 32, 2>(p, s);
    return (int64_t)p.ntx * p.nty > TILE_OCC3_SLOTS ? launch_tile_step_tc<T, 16, 3>(p, s)
                                                    : launch_tile_step_tc<T, 16, 2>(p, s);
}

template <typename T> hipError_t launch_tile_build(const TileIO<T> &p, hipStream_t s) {
    if (p.tc < TILE_TC_MIN || p.tc > TILE_TC_MAX || p.ntx < 3 || p.nty < 3 || p.cap <= 0) return hipErrorInvalidValue;
    if (p.n <= 0) return hipSuccess;
    const unsigned nb = (unsigned)((p.n + 255) / 256);
    hipLaunchKernelGGL((tile_count_kernel<T>), dim3(nb), dim3(256), 0, s, p);
    hipLaunchKernelGGL((tile_scan_kernel<T>), dim3((unsigned)(p.ntx * p.nty)), dim3(TILE_THREADS), 0, s, p);
    hipLaunchKernelGGL((tile_scatter_kernel<T>), dim3(nb), dim3(256), 0, s, p);
    return hipGetLastError();
}

template <typename T> hipError_t launch_tile_unbin(const TileIO<T> &p, hipStream_t s) {
    const int64_t total = (int64_t)p.ntx * p.nty * p.cap;
    const int64_t nbl = (total + 255) / 256;
    const unsigned nb = (unsigned)(nbl < 2048 ? nbl : 2048);
    hipLaunchKernelGGL((tile_unbin_kernel<T>), dim3(nb > 0 ? nb : 1), dim3(256), 0, s, p);
    return hipGetLastError();
}

#if RB_TILE_STAMPS
extern "C" int rb_diag_tile_stamps(unsigned long long *out, int nblocks) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(rb_tile_stamp_buf), sizeof(unsigned long long) * 12 * nblocks);
}
#endif

template hipError_t launch_tile_step<double>(const TileParams<double> &, int, hipStream_t);
template hipError_t launch_tile_step<float>(const TileParams<float> &, int, hipStream_t);
template hipError_t launch_tile_build<double>(const TileIO<double> &, hipStream_t);
template hipError_t launch_tile_build<float>(const TileIO<float> &, hipStream_t);
template hipError_t launch_tile_unbin<double>(const TileIO<double> &, hipStream_t);
template hipError_t launch_tile_unbin<float>(const TileIO<float> &, hipStream_t);

}  // namespace rb
