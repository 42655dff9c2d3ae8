// rb_resident.hip — the resident form of the step (rb_internal.hpp ResParams;
// DESIGN §4.3): sphere worlds on one rank, a window of K reference steps per
// launch.
//
// The step is the reference's: contacts from the step-start positions of
// every body (mj_forward, collision.py:57 / multi_sphere_bounce.py:43), then
// per body gravity, its plane contacts and its sphere partners in ascending
// id, each through compute_collision_impulse_friction (collision.py:7-48) and
// apply_impulse_friction (physics_utils.py:25-49), then the integration
// (collision.py:90-100) — Jacobi across bodies, Gauss-Seidel within one
// (collision.py:72-88).  The per-body arithmetic is rb_body.hpp's, shared
// with the hashed-cell and tile kernels, so every form steps a body
// bit-identically.  What differs is where the step-start data lives and who
// waits for whom:
//
//   hashed cells / tiles: one launch per step; every body's state goes
//     through HBM each step, and the launch boundary orders the steps;
//   here: one launch per window; a single-wave workgroup owns the bodies in
//     one square tile of the plane and keeps their state in registers; each
//     step it imports from its 8 neighbours only what it needs — the
//     positions of their bodies within contact reach R of its tile, and the
//     full state of bodies that crossed into it — as 8-byte granules
//     {tag = step, 32-bit half} the neighbours stored write-through (sc1):
//     the data is its own flag, so a slot waits for its neighbours only.
//     Partners come from the 2 x 2 nearest LDS cells (side >= 2 R) over its
//     own bodies and the imports.
//
// Exactness: every partner of a body lies within R of it, so inside its
// tile's neighbourhood; the slot holds every body within R of its tile (its
// own, and each neighbour's exports: a body is exported to every tile within
// R of it but its owner's), so each body's partner set — and, sorted by id,
// its contact order — equals the hashed forms'.  A body that would need a
// slot outside its old tile's 3 x 3 block (moved more than L - R in a step),
// leaves the grid, or overflows a slot / a publication / the import table,
// and any partner overflow, bad position or timed-out wait, raises ERR_TILE
// with a RES_WHY_* bit and sets the abort word; the commit kernel then leaves
// the id-ordered state at the window start and the host replays the window
// with the hashed forms (rb_capi.hip tile_finish).
#include "rb_device.hpp"
#include "rb_grid.hpp"
#include "rb_internal.hpp"
#include "rb_body.hpp"

// diagnostic build only (RB_RES_STAMPS=1, scripts/res_stamps.py): per
// workgroup s_memrealtime (100 MHz, comparable across XCDs) at the start,
// after the setup, per step (first 16) after the imports arrived and after
// the publication, and at the end
#ifndef RB_RES_STAMPS
#define RB_RES_STAMPS 0
#endif
#if RB_RES_STAMPS
constexpr int RES_NSTAMP = 40;
__device__ unsigned long long rb_res_stamp_buf[1 << 12][RES_NSTAMP];
#define RSTAMP(k)                                                                                  \
    do {                                                                                           \
        unsigned long long r_;                                                                     \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r_)::"memory");             \
        if (threadIdx.x == 0 && blockIdx.x < (1u << 12) && (k) < RES_NSTAMP) rb_res_stamp_buf[blockIdx.x][k] = r_; \
    } while (0)
#else
#define RSTAMP(k) do {} while (0)
#endif

namespace rb {

static_assert(RES_CAP == 64, "one wave per slot: the kernel relies on the wave's lockstep between phases");
static_assert(RES_CAP + RES_NIMP <= 256, "candidate indices are 8-bit");

typedef __attribute__((address_space(1))) unsigned long long res_gu64;
typedef __attribute__((address_space(1))) int32_t res_gi32;

// agent-scope relaxed accesses: global_store / global_load ... sc1 (write-
// through, L1-bypassing; MI355X_MICROARCH.md § visibility)
__device__ __forceinline__ void res_store(unsigned long long *p, unsigned long long v) {
    __hip_atomic_store((res_gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long res_load(const unsigned long long *p) {
    return __hip_atomic_load((res_gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t res_load_i32(const int32_t *p) {
    return __hip_atomic_load((res_gi32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The publication of one slot and step parity (RES_PUB_WORDS granules):
//   [CNT + d]                       direction d's counts: exports | migrants << 16
//   [EXP + (d * EG + g) * EXP_CAP + k]  export k toward d: x y z, id word
//   [MIG + (d * MG + g) * MIG_CAP + k]  migrant k toward d: x y z, q, v, w, id word
// Directions d = (dy + 1) * 3 + (dx + 1) (4: the slot itself, unused); a
// real takes W granules (fp64: low, high half), the id word (id | constant
// type << RES_ID_BITS) one.
template <typename T> struct ResLay {
    static constexpr int W = sizeof(T) == 8 ? 2 : 1;
    static constexpr int EG = 3 * W + 1;
    static constexpr int MR = 13;                    // migrant reals
    static constexpr int MG = MR * W + 1;
    static constexpr int CNT = 0, EXP = 16, MIG = EXP + 9 * EG * RES_EXP_CAP;
    static_assert(MIG + 9 * MG * RES_MIG_CAP <= RES_PUB_WORDS, "publication block");
};
__device__ __forceinline__ unsigned long long res_tagged(unsigned long long tag, uint32_t v) { return tag | v; }
__device__ __forceinline__ void res_put(unsigned long long *p, int stride, double v, unsigned long long tag) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    res_store(p, tag | (uint32_t)u);
    res_store(p + stride, tag | (uint32_t)(u >> 32));
}
__device__ __forceinline__ void res_put(unsigned long long *p, int, float v, unsigned long long tag) {
    res_store(p, tag | __float_as_uint(v));
}
// a real from its granules (g[0], and g[1] for fp64)
template <typename T> __device__ __forceinline__ T res_get(unsigned long long lo, unsigned long long hi) {
    if constexpr (sizeof(T) == 8)
        return __longlong_as_double((long long)(((hi & 0xffffffffull) << 32) | (lo & 0xffffffffull)));
    else return __uint_as_float((uint32_t)lo);
}
// inv(I_world) on first use (rb_body.hpp LazyInvI, value-identical) without
// copies of I and q: I from the LDS constant table, q the caller's register
template <typename T> struct ResInvI {
    const T *I;                                      // ix, iy, iz (LDS)
    const Q4<T> &q;
    bool have = false;
    M3<T> m;
    __device__ __forceinline__ ResInvI(const T *I_, const Q4<T> &q_) : I(I_), q(q_) {}
    __device__ __forceinline__ const M3<T> &get() {
        if (!have) {
            m = np_inv3(inertia_world(V3<T>{I[0], I[1], I[2]}, q));
            have = true;
        }
        return m;
    }
};

// a constant type's (m, I, r) from the kernel's LDS copy of the table (a
// dynamic index into the kernel arguments would copy them to scratch)
template <typename T>
__device__ __forceinline__ void res_type(const T (&tab)[RES_TYPES][5], int ty, T &m, V3<T> &I, T &r) {
    const T *c = tab[ty & (RES_TYPES - 1)];
    m = c[0];
    I = {c[1], c[2], c[3]};
    r = c[4];
}

template <typename T> __device__ __forceinline__ void res_fail(const ResParams<T> &p, int why) {
    atomicOr(p.why, why);
    atomicOr(p.sp.err, ERR_TILE);
    __hip_atomic_store((res_gi32 *)p.abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// inclusive scan over the wave's 64 lanes (DPP, as rb_tiles.hip)
__device__ __forceinline__ int res_wave_scan(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
    return x;
}

// the search cell of a position in a slot's window (tile + R on each side),
// clamped into the window's ncx x ncx cells
template <typename T>
__device__ __forceinline__ int res_cell(T x, T y, T wx0, T wy0, T inv_cs, int ncx) {
    int cx = (int)__builtin_floor((double)((x - wx0) * inv_cs)), cy = (int)__builtin_floor((double)((y - wy0) * inv_cs));
    cx = cx < 0 ? 0 : cx >= ncx ? ncx - 1 : cx;
    cy = cy < 0 ? 0 : cy >= ncx ? ncx - 1 : cy;
    return cy * ncx + cx;
}

template <typename T, int MAXP>
__global__ __launch_bounds__(RES_CAP) __attribute__((amdgpu_waves_per_eu(2, 2)))
void res_step_kernel(const int32_t *err, const int32_t *cnt, ResParams<T> p) {
    using Y = ResLay<T>;
    constexpr int W = Y::W, EG = Y::EG, MG = Y::MG, MR = Y::MR;
    constexpr int NC = RES_CAP + RES_NIMP;          // candidate table: own lanes, then imports
    constexpr int EXP_PRE = 6, MIG_PRE = 1;         // entries per direction read with the counts
    constexpr int NIMM = 16;                        // immigrants per step
    constexpr int NGL = (MG + 1) / 2 > EG ? (MG + 1) / 2 : EG;   // granules a lane reads: an export, or half a migrant
    static_assert(8 * EXP_PRE + 8 * 2 * MIG_PRE == RES_CAP, "lane roles of the import");
    static_assert(NC <= 256, "candidate indices are 8-bit");
    // Every body's state lives in LDS between the phases of a step (registers
    // hold it only while the body is solved): the candidate table's own rows
    // [0, 64) (x, r, id; id -1: a free lane), its q, v, w and constant type.
    // Rows [64, 64 + n_em): this slot's bodies that left it in the last step
    // but stay within R; then the neighbours' exports.
    __shared__ T s_cx[NC], s_cy[NC], s_cz[NC], s_cr[NC];
    __shared__ int32_t s_cid[NC];
    __shared__ T s_q[4][RES_CAP], s_v[3][RES_CAP], s_w[3][RES_CAP];
    __shared__ int32_t s_ty[RES_CAP];
    __shared__ int32_t s_cell[RES_CELLS + 1];       // cell counts, then starts
    __shared__ uint8_t s_sorted[NC];                // candidates sorted by cell
    __shared__ uint8_t s_pl[MAXP][RES_CAP];         // partners in discovery order
    __shared__ T s_mig[NIMM][MR];                   // immigrants' state (x, q, v, w)
    __shared__ int32_t s_migid[NIMM];
    __shared__ int32_t s_nb[9];                     // neighbour slot per direction (-1: none)
    __shared__ int32_t s_cnt[9];                    // the counts read this step
    __shared__ T s_types[RES_TYPES][5];             // constants by type (m, ix, iy, iz, r)

    RSTAMP(0);
    const int lane = threadIdx.x;
    const int nslots = p.ntx * p.nty;
    // XCD-aware: blocks b and b + 8 share an XCD; each XCD takes a contiguous
    // band of slot rows, so most neighbours share its L2 (speed only)
    const int b = (int)blockIdx.x, xq = nslots / (int)N_XCD, xr = nslots % (int)N_XCD, xx = b % (int)N_XCD;
    const int slot = xx * xq + (xx < xr ? xx : xr) + b / (int)N_XCD;
    if (*err & ERR_TILE) return;                    // a window after a failed one: replayed anyway
    const int sx = slot % p.ntx, sy = slot / p.ntx;
    const T tlx = p.ox + (T)sx * p.L, tly = p.oy + (T)sy * p.L;   // the tile's low corner
#pragma unroll
    for (int t = 0; t < RES_TYPES; ++t)
#pragma unroll
        for (int c = 0; c < 5; ++c)
            if (lane == t * 5 + c) s_types[t][c] = p.types[t][c];
    if (lane < 9) {
        const int nx = sx + lane % 3 - 1, ny = sy + lane / 3 - 1;
        s_nb[lane] = (lane == 4 || nx < 0 || ny < 0 || nx >= p.ntx || ny >= p.nty) ? -1 : ny * p.ntx + nx;
    }
    const StepParams<T> &sp = p.sp;
    const uint32_t base = *p.epoch;
    const int n0 = cnt[slot];
    if (n0 > RES_CAP) {                             // (the bin kernel raised it)
        if (lane == 0) res_fail(p, TILE_WHY_CAP);
        return;
    }

    // ---- the own bodies and the window-start imports -----------------------------
    {
        const bool alive = lane < n0;
        int32_t id = -1;
        Snap<T> s0 = {T(0), T(0), T(0), T(0)};
        Q4<T> q = {T(1), T(0), T(0), T(0)};
        V3<T> v = {T(0), T(0), T(0)}, w = {T(0), T(0), T(0)};
        int ty = 0;
        if (alive) {
            id = p.ids[(int64_t)slot * RES_CAP + lane];
            s0 = p.snap[id];
            q = {sp.st.qw()[id], sp.st.qx()[id], sp.st.qy()[id], sp.st.qz()[id]};
            v = {sp.st.vx()[id], sp.st.vy()[id], sp.st.vz()[id]};
            w = {sp.st.wx()[id], sp.st.wy()[id], sp.st.wz()[id]};
            ty = p.type_of[id];
        }
        s_cx[lane] = s0.x; s_cy[lane] = s0.y; s_cz[lane] = s0.z; s_cr[lane] = s0.r; s_cid[lane] = id;
        s_q[0][lane] = q.w; s_q[1][lane] = q.x; s_q[2][lane] = q.y; s_q[3][lane] = q.z;
        s_v[0][lane] = v.x; s_v[1][lane] = v.y; s_v[2][lane] = v.z;
        s_w[0][lane] = w.x; s_w[1][lane] = w.y; s_w[2][lane] = w.z;
        s_ty[lane] = ty;
    }
    __syncthreads();
    int n_em = 0, n_in = 0;
    bool bail = false;
    for (int d = 0; d < 9; ++d) {                   // the neighbours' bodies within R of this tile
        const int nb = s_nb[d];
        if (nb < 0) continue;
        const int nn = cnt[nb];
        const bool has = lane < (nn < RES_CAP ? nn : RES_CAP);
        Snap<T> sn = {T(0), T(0), T(0), T(0)};
        int32_t j = -1;
        if (has) {
            j = p.ids[(int64_t)nb * RES_CAP + lane];
            sn = p.snap[j];
        }
        const bool in = has && sn.x >= tlx - p.R && sn.x < tlx + p.L + p.R && sn.y >= tly - p.R && sn.y < tly + p.L + p.R;
        const uint64_t bal = __ballot(in);
        const int k = n_in + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
        if (in && k < RES_NIMP) {
            s_cx[RES_CAP + k] = sn.x; s_cy[RES_CAP + k] = sn.y; s_cz[RES_CAP + k] = sn.z;
            s_cr[RES_CAP + k] = sn.r; s_cid[RES_CAP + k] = j;
        }
        n_in += __popcll(bal);
    }
    if (n_in > RES_NIMP) {
        if (lane == 0) res_fail(p, RES_WHY_IMPORT);
        bail = true;
    }
    __syncthreads();
    RSTAMP(1);

    // ---- the steps ---------------------------------------------------------------------
    const int ncx = p.ncx, ncell = ncx * ncx;
    for (int t = 0; t < p.K && !bail; ++t) {
        // the tile geometry, re-read each step: hoisted out of the loop, the
        // export bounds of all 9 directions held registers for the whole window
        T L_ = p.L, R_ = p.R, tlx_ = tlx, tly_ = tly;
        asm volatile("" : "+v"(L_), "+v"(R_), "+v"(tlx_), "+v"(tly_));
        const T wx0 = tlx_ - R_, wy0 = tly_ - R_;
        const bool last = t + 1 == p.K;
        if (t > 0) {
            // ---- 1. the imports of step t: each neighbour's counts toward this
            // slot (lanes 0-8), its first EXP_PRE exports (lanes 0-47) and its
            // first migrant (lanes 48-63, two lanes each), in one round trip
            const unsigned long long *src = p.pub + (size_t)(t & 1) * nslots * RES_PUB_WORDS;
            const uint32_t tag = base + (uint32_t)t;
            const int ld = lane < 48 ? lane / EXP_PRE : (lane - 48) / 2;
            const int d = ld < 4 ? ld : ld + 1;
            const int ke = lane % EXP_PRE, mhalf = (lane - 48) & 1;
            const int nb = s_nb[d];
            const unsigned long long *blk = src + (size_t)(nb < 0 ? 0 : nb) * RES_PUB_WORDS;
            const int dc = lane < 9 ? lane : 4;
            const int nbc = s_nb[dc];
            const unsigned long long *pc = src + (size_t)(nbc < 0 ? 0 : nbc) * RES_PUB_WORDS + Y::CNT + (8 - dc);
            // one register array for both roles: an export's EG granules
            // (lanes 0-47) or half of a migrant's MG (lanes 48-63); the rest
            // of the array reads the count again
            const bool role_e = lane < 48;
            const int g0 = role_e ? 0 : mhalf * NGL, gn = role_e ? EG : (MG - g0 < NGL ? MG - g0 : NGL);
            const unsigned long long *pg = role_e ? blk + Y::EXP + (size_t)((8 - d) * EG) * RES_EXP_CAP + ke
                                                  : blk + Y::MIG + (size_t)((8 - d) * MG + g0) * RES_MIG_CAP;
            const int sg = role_e ? RES_EXP_CAP : RES_MIG_CAP;
            unsigned long long gc, gg[NGL];
            auto issue = [&]() {
                gc = res_load(pc);
#pragma unroll
                for (int g = 0; g < NGL; ++g) gg[g] = res_load(g >= gn ? pc : pg + g * sg);
            };
            issue();
            // ---- 2. wait until the counts and the entries they name are fresh
            const bool cneed = lane < 9 && lane != 4 && nbc >= 0;
            int ne = 0, nm = 0;
            uint64_t t0 = 0;
            for (int spin = 0;; ++spin) {
                const bool ok = !cneed || (uint32_t)(gc >> 32) == tag;
                if (__all(ok)) {
                    if (lane < 9) s_cnt[lane] = cneed ? (int32_t)(uint32_t)gc : 0;
                    ne = s_cnt[d] & 0xffff;
                    nm = (int)((uint32_t)s_cnt[d] >> 16);
                    bool eok = true;
                    if (nb >= 0 && (role_e ? ke < ne : 0 < nm)) {
#pragma unroll
                        for (int g = 0; g < NGL; ++g) eok &= g >= gn || (uint32_t)(gg[g] >> 32) == tag;
                    }
                    if (__all(eok)) break;
                }
                if (spin == 0) t0 = __builtin_amdgcn_s_memrealtime();
                __builtin_amdgcn_s_sleep(1);
                if (res_load_i32(p.abort)) { bail = true; break; }
                if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > p.timeout) {
                    if (lane == 0) res_fail(p, RES_WHY_TIMEOUT);
                    bail = true;
                    break;
                }
                issue();
            }
            if (bail) break;
            // ---- 3. exports into the table (after the own emigrants), migrants
            // into free lanes; entries past the first ones read here (rare)
            int pe_d = 0, pm_d = 0, tot_e = 0, tot_m = 0, tot_xe = 0, tot_xm = 0;
#pragma unroll
            for (int dd = 0; dd < 9; ++dd) {
                const int c = s_cnt[dd], e = c & 0xffff, mm = (int)((uint32_t)c >> 16);
                if (dd < d) { pe_d += e; pm_d += mm; }
                tot_e += e; tot_m += mm;
                tot_xe += e > EXP_PRE ? e - EXP_PRE : 0;
                tot_xm += mm > MIG_PRE ? mm - MIG_PRE : 0;
            }
            n_in = tot_e;
            if (n_em + n_in > RES_NIMP || tot_m > NIMM) {
                if (lane == 0) res_fail(p, n_em + n_in > RES_NIMP ? RES_WHY_IMPORT : TILE_WHY_CAP);
                bail = true;
                break;
            }
            auto fin_export = [&](int k, int32_t idw) {      // radius and id from the id word
                s_cr[k] = s_types[((uint32_t)idw >> RES_ID_BITS) & (RES_TYPES - 1)][4];
                s_cid[k] = idw & ((1 << RES_ID_BITS) - 1);
            };
            if (role_e && nb >= 0 && ke < ne) {
                const int k = RES_CAP + n_em + pe_d + ke;
                s_cx[k] = res_get<T>(gg[0], gg[W > 1 ? 1 : 0]);
                s_cy[k] = res_get<T>(gg[W], gg[W > 1 ? W + 1 : W]);
                s_cz[k] = res_get<T>(gg[2 * W], gg[W > 1 ? 2 * W + 1 : 2 * W]);
                fin_export(k, (int32_t)(uint32_t)gg[3 * W]);
            }
            if (!role_e && nb >= 0 && 0 < nm) {
                // this lane's granules g0 .. g0 + gn of the record: whole reals
                // (NGL is even for fp64), the id word last
#pragma unroll
                for (int g = 0; g < NGL; g += W) {
                    const int gi = g0 + g;
                    if (g >= gn) continue;
                    if (gi < MR * W) s_mig[pm_d][gi / W] = res_get<T>(gg[g], gg[W > 1 ? g + 1 : g]);
                    else s_migid[pm_d] = (int32_t)(uint32_t)gg[g];
                }
            }
            // the rest (a direction with more than EXP_PRE exports or MIG_PRE
            // migrants; rare): one granule at a time, its half straight into
            // the 32-bit words of the LDS entry
            for (int u0 = 0; u0 < tot_xe + tot_xm && !bail; u0 += RES_CAP) {
                const int u = u0 + lane;
                const bool isx = u < tot_xe, ism = !isx && u < tot_xe + tot_xm;
                int dd = 0, k = 0, acc = 0, pre2 = 0;
                const int uu = isx ? u : u - tot_xe;
#pragma unroll
                for (int d2 = 0; d2 < 9; ++d2) {
                    const int c = s_cnt[d2], e = c & 0xffff, mm = (int)((uint32_t)c >> 16);
                    const int xn = isx ? (e > EXP_PRE ? e - EXP_PRE : 0) : (mm > MIG_PRE ? mm - MIG_PRE : 0);
                    if (uu >= acc && uu < acc + xn) { dd = d2; k = (isx ? EXP_PRE : MIG_PRE) + uu - acc; }
                    acc += xn;
                }
#pragma unroll
                for (int d2 = 0; d2 < 9; ++d2) {
                    const int c = s_cnt[d2];
                    pre2 += d2 < dd ? (isx ? (c & 0xffff) : (int)((uint32_t)c >> 16)) : 0;
                }
                const int nb2 = s_nb[dd];
                const unsigned long long *b2 = src + (size_t)(nb2 < 0 ? 0 : nb2) * RES_PUB_WORDS;
                const unsigned long long *q0 = isx ? b2 + Y::EXP + (size_t)((8 - dd) * EG) * RES_EXP_CAP + k
                                                   : b2 + Y::MIG + (size_t)((8 - dd) * MG) * RES_MIG_CAP + k;
                const int ng = (isx || ism) ? (isx ? EG : MG) : 0, st2 = isx ? RES_EXP_CAP : RES_MIG_CAP;
                const int kk = isx ? RES_CAP + n_em + pre2 + k : pre2 + k;
                int32_t idw = 0;
                for (int g = 0; g < MG && !bail; ++g) {
                    unsigned long long v2 = 0;
                    uint64_t t1 = 0;
                    for (int spin = 0;; ++spin) {
                        v2 = g < ng ? res_load(q0 + g * st2) : 0;
                        if (__all(g >= ng || (uint32_t)(v2 >> 32) == tag)) break;
                        if (spin == 0) t1 = __builtin_amdgcn_s_memrealtime();
                        __builtin_amdgcn_s_sleep(1);
                        if (res_load_i32(p.abort)) { bail = true; break; }
                        if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t1) > p.timeout) {
                            if (lane == 0) res_fail(p, RES_WHY_TIMEOUT);
                            bail = true;
                            break;
                        }
                    }
                    if (g >= ng) continue;
                    const int rl = g / W, half = g % W;      // real index, half
                    const uint32_t val = (uint32_t)v2;
                    if (isx) {
                        if (rl < 3) {
                            T *dst3 = rl == 0 ? &s_cx[kk] : rl == 1 ? &s_cy[kk] : &s_cz[kk];
                            reinterpret_cast<uint32_t *>(dst3)[half] = val;
                        } else {
                            idw = (int32_t)val;
                        }
                    } else if (rl < MR) {
                        reinterpret_cast<uint32_t *>(&s_mig[kk][rl])[half] = val;
                    } else {
                        s_migid[kk] = (int32_t)val;
                    }
                }
                if (bail) break;
                if (isx) fin_export(kk, idw);
            }
            if (bail) break;
            // immigrants: the r-th (direction-major) into the r-th free lane
            if (tot_m > 0) {
                const bool is_free = s_cid[lane] < 0;
                const uint64_t freem = __ballot(is_free);
                const int r = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(freem >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)freem, 0));
                if (__popcll(freem) < (uint64_t)tot_m) {
                    if (lane == 0) res_fail(p, TILE_WHY_CAP);
                    bail = true;
                    break;
                }
                if (is_free && r < tot_m) {
                    const T *sm_ = s_mig[r];
                    const int32_t idw = s_migid[r];
                    const int ty = (int)((uint32_t)idw >> RES_ID_BITS) & (RES_TYPES - 1);
                    s_cx[lane] = sm_[0]; s_cy[lane] = sm_[1]; s_cz[lane] = sm_[2];
                    s_q[0][lane] = sm_[3]; s_q[1][lane] = sm_[4]; s_q[2][lane] = sm_[5]; s_q[3][lane] = sm_[6];
                    s_v[0][lane] = sm_[7]; s_v[1][lane] = sm_[8]; s_v[2][lane] = sm_[9];
                    s_w[0][lane] = sm_[10]; s_w[1][lane] = sm_[11]; s_w[2][lane] = sm_[12];
                    s_ty[lane] = ty;
                    s_cr[lane] = s_types[ty][4];
                    s_cid[lane] = idw & ((1 << RES_ID_BITS) - 1);
                }
            }
            __syncthreads();
        }
        if (t < 8) RSTAMP(4 + 4 * t);

        // ---- 4. the candidates by cell (LDS counting sort) ---------------------------
        const int ncand = RES_CAP + n_em + n_in;
        for (int c = lane; c <= ncell; c += RES_CAP) s_cell[c] = 0;
        __syncthreads();
        int cl[NC / RES_CAP], rk[NC / RES_CAP];
#pragma unroll
        for (int u = 0; u < NC / RES_CAP; ++u) {
            const int c = lane + u * RES_CAP;
            cl[u] = -1;
            rk[u] = 0;
            if (c < ncand && s_cid[c] >= 0) {
                cl[u] = res_cell(s_cx[c], s_cy[c], wx0, wy0, p.inv_cs, ncx);
                rk[u] = atomicAdd(&s_cell[cl[u]], 1);
            }
        }
        __syncthreads();
        {
            int loc[4], sum = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = lane * 4 + j;
                loc[j] = c < ncell ? s_cell[c] : 0;
                sum += loc[j];
            }
            const int incl = res_wave_scan(sum);
            int ex = incl - sum;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = lane * 4 + j;
                if (c < ncell) s_cell[c] = ex;
                ex += loc[j];
            }
            if (lane == RES_CAP - 1) s_cell[ncell] = incl;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < NC / RES_CAP; ++u)
            if (cl[u] >= 0) s_sorted[s_cell[cl[u]] + rk[u]] = (uint8_t)(lane + u * RES_CAP);
        __syncthreads();

        // ---- 5. one lane per own body (state from LDS): gravity and plane
        // contacts, partners from the 2 x 2 nearest cells solved in ascending
        // id (the canonical order), then the integration
        const int32_t id = s_cid[lane];
        const bool alive = id >= 0;
        const bool rec = last && p.rec && sp.rec_count;
        V3<T> x = {s_cx[lane], s_cy[lane], s_cz[lane]};
        Q4<T> q = {s_q[0][lane], s_q[1][lane], s_q[2][lane], s_q[3][lane]};
        V3<T> v = {s_v[0][lane], s_v[1][lane], s_v[2][lane]};
        V3<T> w = {s_w[0][lane], s_w[1][lane], s_w[2][lane]};
        const T rad = s_cr[lane];
        bool bad = false;
        if (alive) {
            const T *cst = s_types[s_ty[lane]];
            const T m = cst[0];
            ResInvI<T> invI(cst + 1, q);
            const T kimp = impulse_k(m);
            int32_t nrec = 0;
            auto rcd = [&](int32_t partner, int32_t kind, T dist) {
                if (!rec) return;
                if (nrec < sp.maxrec) {
                    const int64_t o = (int64_t)id * sp.maxrec + nrec;
                    sp.rec_partner[o] = partner;
                    sp.rec_kind[o] = kind;
                    sp.rec_dist[o] = dist;
                }
                ++nrec;
            };
            apply_force<T, false, ResInvI<T>>(sp, id, m, invI, v, w);   // (no xfrc: res_eligible)
            for (int pl = 0; pl < sp.n_planes; ++pl) {
                const V3<T> pn = {sp.pn[pl][0], sp.pn[pl][1], sp.pn[pl][2]};
                const V3<T> pp = {sp.pp[pl][0], sp.pp[pl][1], sp.pp[pl][2]};
                Contact<T> con;
                if (!plane_sphere(pn, pp, x, rad, con)) continue;
                rcd(-1 - pl, 0, con.dist);
                solve_contact(sp, con, x, con.frame, m, kimp, invI, v, w);
            }
            const T fx = (x.x - wx0) * p.inv_cs, fy = (x.y - wy0) * p.inv_cs;
            const int cx = (int)__builtin_floor((double)fx), cy = (int)__builtin_floor((double)fy);
            const int c0 = fx - (T)cx >= T(0.5) ? cx : cx - 1;
            const int r1 = fy - (T)cy >= T(0.5) ? cy + 1 : cy - 1;
            const int lo = c0 < 0 ? 0 : c0, hi = c0 + 1 >= ncx ? ncx - 1 : c0 + 1;
            int np_ = 0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int rr = h == 0 ? cy : r1;
                if (rr < 0 || rr >= ncx || lo > hi) continue;
                const int a0 = s_cell[rr * ncx + lo], a1 = s_cell[rr * ncx + hi + 1];
                for (int k = a0; k < a1; ++k) {
                    const int c = s_sorted[k];
                    if (s_cid[c] == id) continue;
                    if (sphere_sphere_hit(x, rad, V3<T>{s_cx[c], s_cy[c], s_cz[c]}, s_cr[c])) {
                        if (np_ < MAXP) s_pl[np_][lane] = (uint8_t)c;
                        ++np_;
                    }
                }
            }
            if (np_ > MAXP) {
                res_fail(p, TILE_WHY_PARTNERS);
                bad = true;
                np_ = MAXP;
            }
            int32_t prev = -1;
            for (int a = 0; a < np_; ++a) {
                int c = 0;
                int32_t j = INT32_MAX;
                for (int e = 0; e < np_; ++e) {
                    const int ce = s_pl[e][lane];
                    const int32_t ie = s_cid[ce];
                    if (ie > prev && ie < j) { j = ie; c = ce; }
                }
                prev = j;
                const V3<T> cj = {s_cx[c], s_cy[c], s_cz[c]};
                const T rj = s_cr[c];
                Contact<T> con;
                V3<T> nrm;
                if (id < j) {                            // this body is geom1
                    sphere_sphere(x, rad, cj, rj, con);
                    nrm = sp.oriented ? V3<T>{-con.frame.x, -con.frame.y, -con.frame.z} : con.frame;
                } else {
                    sphere_sphere(cj, rj, x, rad, con);
                    nrm = con.frame;
                }
                rcd(j, 16, con.dist);
                solve_contact(sp, con, x, nrm, m, kimp, invI, v, w);
            }
            if (rec) sp.rec_count[id] = nrec;
            Q4<T> qn;
            integrate_pose(x, qn, q, v, w, sp.dt);
            q = qn;
        }
        if (__any(bad)) { bail = true; break; }
        if (t < 8) RSTAMP(6 + 4 * t);
        if (last) {
            // the window's end state (committed by res_commit_kernel if no slot failed)
            if (alive) {
                p.out_snap[id] = Snap<T>{x.x, x.y, x.z, rad};
                T *o = p.out_st;
                const int64_t S = sp.st.S;
                o[0 * S + id] = q.w; o[1 * S + id] = q.x; o[2 * S + id] = q.y; o[3 * S + id] = q.z;
                o[4 * S + id] = v.x; o[5 * S + id] = v.y; o[6 * S + id] = v.z;
                o[7 * S + id] = w.x; o[8 * S + id] = w.y; o[9 * S + id] = w.z;
            }
            break;
        }

        // ---- 6. the new owner and the recipients of every body, published with
        // tag t + 1: exports (within R of another tile), migrants (into a
        // neighbour's tile), and own emigrants kept for this slot's next step
        uint32_t ef = 0;                                 // export directions (4: this slot)
        int dm = -1;                                     // migration direction
        if (alive) {
            int why = 0;
            const T fxt = (x.x - p.ox) * p.inv_L, fyt = (x.y - p.oy) * p.inv_L;
            if (!(absval(fxt) < T(1 << 29) && absval(fyt) < T(1 << 29) && absval(x.z) < T(1e12))) {
                why = TILE_WHY_DOMAIN;
            } else {
                const int ntx_ = (int)__builtin_floor((double)fxt), nty_ = (int)__builtin_floor((double)fyt);
                if (ntx_ < 0 || nty_ < 0 || ntx_ >= p.ntx || nty_ >= p.nty) why = RES_WHY_GRID;
                // every tile within R of the body must be a neighbour of this one
                else if (!(x.x >= tlx_ - L_ + R_ && x.x < tlx_ + T(2) * L_ - R_ && x.y >= tly_ - L_ + R_ &&
                           x.y < tly_ + T(2) * L_ - R_)) why = RES_WHY_MOVE;
                else {
                    const int ddx = ntx_ - sx, ddy = nty_ - sy;
                    if (ddx != 0 || ddy != 0) dm = (ddy + 1) * 3 + (ddx + 1);
#pragma unroll
                    for (int dd = 0; dd < 9; ++dd) {
                        const int ux = sx + dd % 3 - 1, uy = sy + dd / 3 - 1;
                        if (ux < 0 || uy < 0 || ux >= p.ntx || uy >= p.nty || dd == dm || (dd == 4 && dm < 0)) continue;
                        const T ulx = p.ox + (T)ux * L_, uly = p.oy + (T)uy * L_;
                        if (x.x >= ulx - R_ && x.x < ulx + L_ + R_ && x.y >= uly - R_ && x.y < uly + L_ + R_)
                            ef |= 1u << dd;
                    }
                }
            }
            if (why) {
                res_fail(p, why);
                bad = true;
            }
        }
        if (__any(bad)) { bail = true; break; }
        const size_t par1 = (size_t)((t + 1) & 1);
        unsigned long long *dst = p.pub + (par1 * nslots + slot) * RES_PUB_WORDS;
        const unsigned long long tg1 = (unsigned long long)(base + (uint32_t)(t + 1)) << 32;
        const uint32_t idw = alive ? ((uint32_t)id | ((uint32_t)s_ty[lane] << RES_ID_BITS)) : 0u;
        int my_ne = 0, my_nm = 0, em_new = 0;
        bool over = false;
        // (the table rows of this step are read no more: the wave is past its search)
#pragma unroll 1
        for (int dd = 0; dd < 9; ++dd) {
            const bool fe = alive && ((ef >> dd) & 1u), fm = alive && dm == dd;
            const uint64_t be = __ballot(fe), bm = __ballot(fm);
            const int ke2 = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(be >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)be, 0));
            const int km2 = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0));
            const int ce = __popcll(be), cm = __popcll(bm);
            if (lane == dd) { my_ne = ce; my_nm = cm; }
            if (dd == 4) {
                // own emigrants within R: candidates of this slot's next step
                em_new = ce;
                if (fe && ke2 < RES_NIMP) {
                    s_cx[RES_CAP + ke2] = x.x; s_cy[RES_CAP + ke2] = x.y; s_cz[RES_CAP + ke2] = x.z;
                    s_cr[RES_CAP + ke2] = rad; s_cid[RES_CAP + ke2] = id;
                }
                continue;
            }
            over |= ce > RES_EXP_CAP || cm > RES_MIG_CAP;
            if (fe && ke2 < RES_EXP_CAP) {
                unsigned long long *o = dst + Y::EXP + (size_t)(dd * EG) * RES_EXP_CAP + ke2;
                res_put(o, RES_EXP_CAP, x.x, tg1);
                res_put(o + W * RES_EXP_CAP, RES_EXP_CAP, x.y, tg1);
                res_put(o + 2 * W * RES_EXP_CAP, RES_EXP_CAP, x.z, tg1);
                res_store(o + 3 * W * RES_EXP_CAP, tg1 | idw);
            }
            if (fm && km2 < RES_MIG_CAP) {
                unsigned long long *o = dst + Y::MIG + (size_t)(dd * MG) * RES_MIG_CAP + km2;
                const T rs[MR] = {x.x, x.y, x.z, q.w, q.x, q.y, q.z, v.x, v.y, v.z, w.x, w.y, w.z};
#pragma unroll
                for (int r = 0; r < MR; ++r) res_put(o + r * W * RES_MIG_CAP, RES_MIG_CAP, rs[r], tg1);
                res_store(o + MR * W * RES_MIG_CAP, tg1 | idw);
            }
        }
        if (lane < 9 && lane != 4) res_store(dst + Y::CNT + lane, tg1 | (uint32_t)(my_ne | (my_nm << 16)));
        if (over || em_new > RES_NIMP) {
            if (lane == 0) res_fail(p, over ? RES_WHY_PUB : RES_WHY_IMPORT);
            bail = true;
            break;
        }
        n_em = em_new;
        // the own rows for the next step; an emigrant frees its lane
        const bool stays = alive && dm < 0;
        s_cx[lane] = x.x; s_cy[lane] = x.y; s_cz[lane] = x.z; s_cid[lane] = stays ? id : -1;
        s_q[0][lane] = q.w; s_q[1][lane] = q.x; s_q[2][lane] = q.y; s_q[3][lane] = q.z;
        s_v[0][lane] = v.x; s_v[1][lane] = v.y; s_v[2][lane] = v.z;
        s_w[0][lane] = w.x; s_w[1][lane] = w.y; s_w[2][lane] = w.z;
        __syncthreads();
        if (t < 8) RSTAMP(7 + 4 * t);
    }
    RSTAMP(2);
}

// ---- binning and commit ----------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void res_bin_kernel(ResParams<T> p, int64_t n) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= n) return;
    const Snap<T> sn = p.snap[b];
    const T fx = (sn.x - p.ox) * p.inv_L, fy = (sn.y - p.oy) * p.inv_L;
    if (!(absval(fx) < T(1 << 29) && absval(fy) < T(1 << 29))) {
        atomicOr(p.why, TILE_WHY_DOMAIN);
        atomicOr(p.sp.err, ERR_TILE);
        return;
    }
    const int32_t tx = (int32_t)__builtin_floor((double)fx), ty = (int32_t)__builtin_floor((double)fy);
    if (tx < 0 || ty < 0 || tx >= p.ntx || ty >= p.nty) {        // outside the grid: a new fit
        atomicOr(p.why, RES_WHY_GRID);
        atomicOr(p.sp.err, ERR_TILE);
        return;
    }
    const int64_t slot = (int64_t)ty * p.ntx + tx;
    const int32_t k = atomicAdd(const_cast<int32_t *>(p.cnt) + slot, 1);
    if (k < RES_CAP) {
        const_cast<int32_t *>(p.ids)[slot * RES_CAP + k] = (int32_t)b;
    } else if (k == RES_CAP) {
        atomicOr(p.why, TILE_WHY_CAP);
        atomicOr(p.sp.err, ERR_TILE);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void res_commit_kernel(ResCommit<T> p) {
    const bool ok = !(*p.err & ERR_TILE);
    const int64_t stride = (int64_t)gridDim.x * 256;
    if (ok) {
        for (int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x; b < p.n; b += stride) {
            p.snap[b] = p.out_snap[b];
#pragma unroll
            for (int d = 0; d < 10; ++d) p.st.row(d)[b] = p.out_st[d * p.S + b];
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *p.epoch += (uint32_t)p.K + 1u;
        *p.abort = 0;
        if (ok) *p.commits += 1;
    }
}

// ---- launchers ----------------------------------------------------------------
template <typename T> hipError_t launch_res_bin(const ResParams<T> &p, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL((res_bin_kernel<T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, n);
    return hipGetLastError();
}
template <typename T> hipError_t launch_res_step(const ResParams<T> &p, int maxp, hipStream_t s) {
    if (p.ntx < 1 || p.nty < 1 || p.K < 1 || !(p.L > 0) || p.ncx < 1 || p.ncx * p.ncx > RES_CELLS) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(p.ntx * p.nty)), block(RES_CAP);
    if (maxp > 16) hipLaunchKernelGGL((res_step_kernel<T, 32>), grid, block, 0, s, p.sp.err, p.cnt, p);
    else hipLaunchKernelGGL((res_step_kernel<T, 16>), grid, block, 0, s, p.sp.err, p.cnt, p);
    return hipGetLastError();
}
template <typename T> hipError_t launch_res_commit(const ResCommit<T> &p, hipStream_t s) {
    const int64_t nb = (p.n + 255) / 256;
    hipLaunchKernelGGL((res_commit_kernel<T>), dim3((unsigned)(nb < 1024 ? (nb > 0 ? nb : 1) : 1024)), dim3(256), 0, s, p);
    return hipGetLastError();
}

int res_blocks_per_cu(int f64, int maxp) {
    int nb = 0;
    hipError_t r;
    if (f64) r = maxp > 16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, res_step_kernel<double, 32>, RES_CAP, 0)
                           : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, res_step_kernel<double, 16>, RES_CAP, 0);
    else r = maxp > 16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, res_step_kernel<float, 32>, RES_CAP, 0)
                       : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, res_step_kernel<float, 16>, RES_CAP, 0);
    return r == hipSuccess ? nb : 0;
}

#if RB_RES_STAMPS
extern "C" int rb_diag_res_stamps(unsigned long long *out, int nblocks) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(rb_res_stamp_buf), sizeof(unsigned long long) * RES_NSTAMP * nblocks);
}
#endif

template hipError_t launch_res_bin<double>(const ResParams<double> &, int64_t, hipStream_t);
template hipError_t launch_res_bin<float>(const ResParams<float> &, int64_t, hipStream_t);
template hipError_t launch_res_step<double>(const ResParams<double> &, int, hipStream_t);
template hipError_t launch_res_step<float>(const ResParams<float> &, int, hipStream_t);
template hipError_t launch_res_commit<double>(const ResCommit<double> &, hipStream_t);
template hipError_t launch_res_commit<float>(const ResCommit<float> &, hipStream_t);

}  // namespace rb
