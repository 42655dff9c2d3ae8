// rb_kernels.hip — the hot path on gfx950.
//
// One launch per simulation step (rb::step_kernel), 64-thread workgroups
// (one wave):
//   K1 contact generation  — plane-sphere / plane-box corners against the
//      static planes; sphere-sphere against the step-start snapshot through
//      a spatial hash of cells (2 x 2 x 2 nearest cells).  Partners go to a
//      per-body list in LDS in ascending body id = the canonical
//      Gauss-Seidel order (SURVEY §7 hard part 1).  Small scenes search
//      cooperatively (8 lanes per body, one per cell), large ones one lane
//      per body.
//   K2 impulse solve       — per contact, in list order:
//      compute_collision_impulse_friction (collision.py:7-48) then
//      apply_impulse_friction (physics_utils.py:25-49);
//   K3 integrate           — x += v dt, q += 0.5 (0,w)*q dt, normalise
//      (collision.py:90-95): state written in place, the new position into
//      the next snapshot;
//   and the next step's broadphase: the body inserts its id into the next
//   table (a newer generation, rb_internal.hpp Table: nothing is cleared).
//   Two tables and two snapshots alternate, so a step reads only data no
//   thread of the same launch writes: Jacobi across bodies, exactly as
//   multi_sphere_bounce.py:43-46 (one mj_forward per step).
#include "rb_device.hpp"

// diagnostic build only: per-wave s_memtime stamps at phase boundaries.
// One unit keeps them (the fp64 wide unit): the host-side name of the
// buffer must be unique in the library
#ifndef RB_STAMPS
#define RB_STAMPS 0
#endif
#if RB_STAMPS && !(defined(RB_WIDE_UNIT) && RB_WIDE_UNIT == 1 && defined(RB_INST) && RB_INST == 1)
#undef RB_STAMPS
#define RB_STAMPS 0
#endif
#if RB_STAMPS
__device__ unsigned long long rb_stamp_buf[1 << 16][16];
#define STAMP(k)                                                                                  \
    do {                                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        unsigned long long t_;                                                                    \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        if (tid == 0 && blockIdx.x < (1u << 16)) rb_stamp_buf[blockIdx.x][k] = t_;                \
        if (k == 0 || k == 6) { /* the constant-rate clock too, comparable across XCDs */            \
            unsigned long long r_;                                                                \
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r_)::"memory");        \
            if (tid == 0 && blockIdx.x < (1u << 16)) rb_stamp_buf[blockIdx.x][k == 0 ? 12 : 13] = r_; \
        }                                                                                         \
    } while (0)
#else
#define STAMP(k) do {} while (0)
#endif

#include "rb_boxes.hpp"
#include "rb_grid.hpp"
#include "rb_halo.hpp"
#include "rb_internal.hpp"
#include "rb_body.hpp"

// diagnostic builds only (scripts/ablate.py): 1 = skip the sphere-sphere
// broadphase, 2 = skip the world-inertia inverse (identity), 3 = empty
// kernel (launch floor), 4 = search only (no body update), 0 = product
#ifndef RB_ABLATE
#define RB_ABLATE 0
#endif

namespace rb {

template <typename T>
__global__ __launch_bounds__(256) void insert_kernel(InsertParams<T> p) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= p.count) return;
    const int64_t id = p.first + k;
    if (id >= p.skip_lo && id < p.skip_hi) return;
    insert_id(p.grid, p.tab, p.err, p.snap[id], (uint32_t)id | (p.kind[id] != 0 ? BOX_FLAG : 0u), *p.tab.gen);
}

// Candidate test shared by every search form: true if the candidate with
// snapshot s and tagged id tj is a partner of body i — for two spheres the
// sphere-sphere contact test, for a box-involved pair overlapping bounding
// spheres (the narrowphase then decides; oracle gen_contacts does the
// same).  Only the box kernel (BOXES) takes such a pair; the sphere step
// kernels mark the body deferred to it (box worlds, sharded or not: p.defer_q;
// a sharded world's exchange carries the boxes' orientations).
template <typename T, bool BOXES>
__device__ __forceinline__ bool candidate_hit(const StepParams<T> &p, int32_t i, int32_t kind, V3<T> x, T rad, T bi,
                                              uint32_t tj, const Snap<T> &s, bool &defer) {
    const int32_t j = (int32_t)(tj & ~BOX_FLAG);
    if (j == i) return false;
    const V3<T> cj = {s.x, s.y, s.z};
    if (kind != 0 || (tj & BOX_FLAG)) {
        const V3<T> dd = {x.x - cj.x, x.y - cj.y, x.z - cj.z};
        const bool near = sqroot(mj_dot(dd, dd)) <= bi + s.r;
        if (BOXES) return near;
        if (near) {
            if (p.defer_q) defer = true;
            else atomicOr(p.err, ERR_UNSUPPORTED);
        }
        return false;
    }
    return sphere_sphere_hit(x, rad, cj, s.r);
}

// K1, one lane per body (rb_grid.hpp search_buckets with the main law's
// candidate test).
template <typename T, int MAXP, bool BOXES>
__device__ __forceinline__ int32_t search_partners(const StepParams<T> &p, int32_t i, int32_t kind, V3<T> x,
                                                   T rad, T bi, int32_t *s_id, int tid, uint32_t gen, bool &defer) {
    // the box kernel also runs in cooperative worlds (a hash per cell)
    constexpr int L = BOXES ? LAYOUT_ANY : LAYOUT_LINEAR;
    return search_buckets<T, MAXP, L>(p, i, x, s_id, tid, gen, [&](uint32_t tj, const Snap<T> &s) {
        return candidate_hit<T, BOXES>(p, i, kind, x, rad, bi, tj, s, defer);
    });
}

// K1, wide one-lane form (rb_grid.hpp search_buckets_wide)
template <typename T, int MAXP, bool BOXES, typename Overlap>
__device__ __forceinline__ int32_t search_partners_wide(const StepParams<T> &p, int32_t i, int32_t kind, V3<T> x,
                                                        T rad, T bi, int32_t *s_id, uint32_t *s_cand, uint8_t *s_didx,
                                                        Snap<T> *s_hpos, int tid, uint32_t gen, bool &defer,
                                                        Overlap overlap) {
    return search_buckets_wide<T, MAXP>(
        p, i, x, s_id, s_cand, s_didx, s_hpos, tid, gen,
        [&](uint32_t tj, const Snap<T> &s) { return candidate_hit<T, BOXES>(p, i, kind, x, rad, bi, tj, s, defer); },
        overlap);
}

// K1 for small scenes: G lanes per body, lane k of the group owns neighbour
// cell k.  Its header (count, first 2 ids) and first RB_QSPEC slot snapshots are
// loaded together (slots past the count are stale and ignored), and while
// they are in flight the lane evaluates the body's inverse world inertia
// (pre, if PRE).  Hits become a bitmask over the bucket slots; a group prefix sum
// (shuffles) places them — id and snapshot — in LDS, and the group
// rank-sorts them by body id into s_id / s_pos.  Same contact set and order
// as search_partners.
template <typename T, int MAXP, int G, bool BOXES, int RL, typename Overlap>
__device__ __forceinline__ int32_t search_coop(const StepParams<T> &p, bool active, int32_t i, int32_t kind,
                                               V3<T> x, T rad, T bi, int32_t *s_id, Snap<T> *s_pos, int32_t *t_id,
                                               Snap<T> *t_pos, int slot, int k, int lane, uint32_t gen,
                                               bool &defer, Overlap overlap) {
    static_assert(G == 8, "one lane per neighbour cell");
    constexpr int NB = STEP_BLOCK / G;
    constexpr int QB = RB_QBATCH;
    constexpr int QS = RB_QSPEC;                 // slots loaded before the count is known
    int32_t cx = 0, cy = 0, cz = 0, sx = 1, sy = 1, sz = 1;
    bool ok = active;
    if (active && !neighbourhood(p, x, cx, cy, cz, sx, sy, sz)) {
        if (k == 0) atomicOr(p.err, ERR_DOMAIN);
        ok = false;
    }
    const uint32_t b = bucket_of(cx + ((k & 1) ? sx : 0), cy + ((k & 2) ? sy : 0), cz + ((k & 4) ? sz : 0),
                                 p.grid);
    const int64_t base = (int64_t)b * LINE_WORDS;      // slot snapshots: slot s at base + s
    [[maybe_unused]] const int tid = lane;   // STAMP
    STAMP(8);
    // loaded unconditionally (b is a valid bucket for every lane) and the
    // count clamped only after overlap(): a use inside a branch would make
    // the wave wait for the loads before that work starts
    const int rl = RL >= 0 ? RL : grid_rl(p.grid.super);   // heads per line: cooperative worlds 1 (rb_capi.hip)
    const uint4 id4 = bucket_head(p.cur, b, rl);
    Snap<T> p4[QS > 0 ? QS : 1];                  // (RB_QSPEC=0: a diagnostic build)
#pragma unroll
    for (int u = 0; u < QS; ++u) p4[u] = p.cur.pos[base + u];
    __builtin_amdgcn_sched_barrier(0);            // the bucket loads issue before the body work
    overlap();                                    // body work under the bucket loads
    int32_t c = !ok ? 0 : head_count(id4, gen);
    STAMP(9);
    const int gbase = lane & ~(G - 1);
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const uint32_t bj = (uint32_t)__shfl((int)b, gbase + j);
        if (j < k && bj == b) c = 0;                  // bucket already visited by a lower cell
    }
    uint32_t mask = 0;
#pragma unroll
    for (int u = 0; u < QS; ++u)
        if (u < c && candidate_hit<T, BOXES>(p, i, kind, x, rad, bi, bucket_id(p.cur, b, id4, u, rl), p4[u], defer)) mask |= 1u << u;
    for (int s0 = QS; s0 < c; s0 += QB) {
        uint32_t tj[QB];
        Snap<T> sn[QB];
#pragma unroll
        for (int u = 0; u < QB; ++u) {
            if (s0 + u >= c) break;                   // stay inside this bucket's slots
            tj[u] = bucket_id(p.cur, b, id4, s0 + u, rl);
            sn[u] = p.cur.pos[base + s0 + u];
        }
#pragma unroll
        for (int u = 0; u < QB; ++u)
            if (s0 + u < c && candidate_hit<T, BOXES>(p, i, kind, x, rad, bi, tj[u], sn[u], defer)) mask |= 1u << (s0 + u);
    }
    // rare: ids past a full bucket (rb_grid.hpp spill_scan), counted here,
    // placed after the slot hits below (id-indexed snapshots: no slot copy)
    int32_t hs = 0;
    const bool spl = c > 0 && head_spilled(id4, gen);
    if (spl)
        spill_scan(p.cur, gen, b, [&](uint32_t t) {
            if (candidate_hit<T, BOXES>(p, i, kind, x, rad, bi, t, p.snap_cur[CHK(t & ~BOX_FLAG, p.n_global)], defer)) ++hs;
        });
    STAMP(10);
    if (p.defer_q) {                              // any lane of the group: the body is deferred
        int dv = defer ? 1 : 0;
        dv |= __shfl_xor(dv, 1);
        dv |= __shfl_xor(dv, 2);
        dv |= __shfl_xor(dv, 4);
        defer = dv != 0;
    }
    const int h = __popc(mask) + hs;
    int pre_n = 0, total = 0;
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const int hj = __shfl(h, gbase + j);
        total += hj;
        if (j < k) pre_n += hj;
    }
    if (total > MAXP && k == 0) atomicOr(p.err, ERR_PARTNER_OVERFLOW);
    int o = pre_n;
#pragma unroll
    for (int u = 0; u < QS; ++u) {
        if (!((mask >> u) & 1u)) continue;
        if (o < MAXP) {
            t_id[slot * MAXP + o] = (int32_t)(bucket_id(p.cur, b, id4, u, rl) & ~BOX_FLAG);
            t_pos[slot * MAXP + o] = p4[u];
        }
        ++o;
    }
    for (uint32_t rest = mask & ~((1u << QS) - 1u); rest; rest &= rest - 1) {
        const int sl = __builtin_ctz(rest);
        if (o < MAXP) {                               // re-read: L1-hot from the batch above
            t_id[slot * MAXP + o] = (int32_t)(bucket_id(p.cur, b, id4, sl, rl) & ~BOX_FLAG);
            t_pos[slot * MAXP + o] = p.cur.pos[base + sl];
        }
        ++o;
    }
    if (hs)
        spill_scan(p.cur, gen, b, [&](uint32_t t) {
            const Snap<T> sn = p.snap_cur[CHK(t & ~BOX_FLAG, p.n_global)];
            bool d2 = false;
            if (!candidate_hit<T, BOXES>(p, i, kind, x, rad, bi, t, sn, d2)) return;
            if (o < MAXP) {
                t_id[slot * MAXP + o] = (int32_t)(t & ~BOX_FLAG);
                t_pos[slot * MAXP + o] = sn;
            }
            ++o;
        });
    __syncthreads();
    STAMP(11);
    const int tot = total < MAXP ? total : MAXP;
    for (int qq = k; qq < tot; qq += G) {
        const int32_t id = t_id[slot * MAXP + qq];
        int r = 0;
        for (int j = 0; j < tot; ++j) r += t_id[slot * MAXP + j] < id;
        s_id[r * NB + slot] = id;
        s_pos[r * NB + slot] = t_pos[slot * MAXP + qq];
    }
    __syncthreads();
    return tot;
}

// Per-body inputs of K2, loaded by the cooperative form before the search
// (their latency hides under it) and by the one-lane form after it (fewer
// registers live across the search).
template <typename T> struct BodyIn {
    Q4<T> q;
    V3<T> v, w;
    T m;
    V3<T> I;
};
template <typename T>
__device__ __forceinline__ BodyIn<T> load_body(const BodyState<T> &st, const BodyConsts<T> &cs, int32_t l, int32_t i) {
    BodyIn<T> b;
    b.q = {st.qw()[l], st.qx()[l], st.qy()[l], st.qz()[l]};
    b.v = {st.vx()[l], st.vy()[l], st.vz()[l]};
    b.w = {st.wx()[l], st.wy()[l], st.wz()[l]};
    // diagnostic (RB_ABLATE 8): every body reads body 0's constants (a
    // scene of identical bodies stays bit-exact) — the cost of the per-body
    // constant loads
    const int32_t ci = RB_ABLATE == 8 ? 0 : i;
    b.m = cs.mass()[ci];
    b.I = {cs.ix()[ci], cs.iy()[ci], cs.iz()[ci]};
    return b;
}
template <typename T> __device__ __forceinline__ BodyIn<T> load_body(const StepParams<T> &p, int32_t l, int32_t i) {
    return load_body(p.st, p.cs, l, i);
}

// The fields a step's first loads need (the body's snapshot, kind, state and
// constants).  The step kernels take them as leading scalar arguments, which
// gfx950 preloads into SGPRs as the waves launch (the units are built with
// -amdgpu-kernarg-preload-count), so their first loads wait for no scalar
// load of the parameter block (measured 0.27 us per launch in
// scripts/preload_probe.hip); the box kernel takes them from the block.
template <typename T> struct Lead {
    const Snap<T> *snap_cur;
    BodyState<T> st;
    BodyConsts<T> cs;
    int32_t n_local, lo;
    __device__ static Lead of(const StepParams<T> &p) { return Lead{p.snap_cur, p.st, p.cs, p.n_local, p.lo}; }
};
#define LEAD_ARGS(p) (p).snap_cur, (p).st.base, (p).st.S, (p).cs.base, (p).cs.Npad, (p).cs.kind, (p).n_local, (p).lo

#ifndef RB_SOLVE_PIPE
#define RB_SOLVE_PIPE 1
#endif
// batches of partner snapshots in flight ahead of the solve (the helper-wave
// wide form only: its register budget has room for a second batch)
#ifndef RB_SOLVE_DEPTH
#define RB_SOLVE_DEPTH 1
#endif

// Everything after the contact search for one body (lane): gravity (unless
// already applied: forced), the Gauss-Seidel solves in canonical order,
// integration, next-step insert.
// The sorted partner list: ids at pid[u * stride] (an LDS column, or the
// split form's per-slot list in HBM); snapshots (PM, partner mode) at
// ppos[u * stride] (LDS, PM = 1: cooperative form), at ppos[d * stride] for
// the discovery index d = pdidx[u * stride] < WIDE_HPOS (LDS, PM = 2: wide
// form) or gathered from the step-start snapshot (PM = 0, and PM = 2 past
// WIDE_HPOS).  A template flag, so LDS accesses stay ds_read (no flat loads).
template <typename T, int PM, bool BOXES = false, int SDEPTH = 1>
__device__ __forceinline__ void body_update(const StepParams<T> &p, int32_t l, int32_t i, V3<T> x, int32_t kind,
                                            V3<T> sz, T bi, const BodyIn<T> &in, bool forced, LazyInvI<T> &invI,
                                            int32_t np_, const int32_t *pid, int64_t stride, const Snap<T> *ppos,
                                            int tid, int32_t *cell, uint32_t gen_next, T *poly = nullptr,
                                            int ps = 0, const uint8_t *pdidx = nullptr, int32_t nrec_in = 0,
                                            bool planes_done = false) {
    const Q4<T> q = in.q;
    V3<T> v = in.v;
    V3<T> w = in.w;
    const T m = in.m;

    // ---- a4: gravity / applied force (collision.py:66-70) ------------------
    if (!forced) apply_force(p, l, m, invI, v, w);
    const T k = impulse_k(m);

    STAMP(3);
    int32_t nrec = nrec_in;
    // ---- K2: plane contacts, plane order -------------------------------------
    // (a sphere's already solved by the helper wave when planes_done)
    if (kind == 0 && !planes_done) {
        for (int pl = 0; pl < p.n_planes; ++pl) {
            const V3<T> pn = {p.pn[pl][0], p.pn[pl][1], p.pn[pl][2]};
            const V3<T> pp = {p.pp[pl][0], p.pp[pl][1], p.pp[pl][2]};
            Contact<T> con;
            if (!plane_sphere(pn, pp, x, sz.x, con)) continue;
            record(p, l, nrec, -1 - pl, 0, con.dist);
            solve_contact(p, con, x, con.frame, m, k, invI, v, w);
        }
    }
    M3<T> M;                                       // box orientation (mj_kinematics of the free joint)
    if (kind != 0) M = mj_body_mat(q);
    if (kind != 0 && !planes_done) {               // (a box's corners likewise)
        for (int pl = 0; pl < p.n_planes; ++pl) {
            const V3<T> pn = {p.pn[pl][0], p.pn[pl][1], p.pn[pl][2]};
            const V3<T> dif = {x.x - p.pp[pl][0], x.y - p.pp[pl][1], x.z - p.pp[pl][2]};
            const T dist = mj_dot(dif, pn);
            int cnt = 0;
            for (int c = 0; c < 8 && cnt < 4; ++c) {
                Contact<T> con;
                if (!plane_box_corner(pn, x, dist, M, sz, c, con)) continue;
                ++cnt;
                record(p, l, nrec, -1 - pl, 1 + c, con.dist);
                solve_contact(p, con, x, con.frame, m, k, invI, v, w);
            }
        }
    }

    // ---- K2: sphere partners in ascending id order ---------------------------
    // (partner snapshots fetched PB at a time; the solve itself is the
    // reference's sequential Gauss-Seidel).  The box kernel takes them one at
    // a time: each unrolled copy of the loop body inlines the box
    // narrowphase (4 copies made the kernel 169 KB)
    constexpr int PB = BOXES ? 1 : 4;
    auto fetch = [&](int s0, int32_t (&jj)[PB], Snap<T> (&pe)[PB]) {
#pragma unroll
        for (int u = 0; u < PB; ++u)
            if (s0 + u < np_) jj[u] = pid[CHK((s0 + u) * stride, 32 * stride)];
#pragma unroll
        for (int u = 0; u < PB; ++u) {
            if (s0 + u >= np_) continue;
            if constexpr (PM == 1) {
                pe[u] = ppos[(s0 + u) * stride];
            } else if constexpr (PM == 2) {
                const int d = pdidx[(s0 + u) * stride];
                pe[u] = d < WIDE_HPOS ? ppos[d * stride] : xld(p.snap_cur + CHK(jj[u], p.n_global));
            } else {
                pe[u] = xld(p.snap_cur + CHK(jj[u], p.n_global));
            }
        }
    };
    // sphere kernels (RB_SOLVE_PIPE): the next batch's snapshots load under
    // this batch's solves — a body with many partners (C4's pile-ups: up to
    // 28) otherwise waits one round trip per PB partners re-read from memory
    [[maybe_unused]] int32_t jn[PB], jn2[PB];
    [[maybe_unused]] Snap<T> sn_next[PB], sn_next2[PB];
    constexpr bool pipe = !BOXES && RB_SOLVE_PIPE && PM != 1;   // (the cooperative form: LDS only)
    constexpr bool deep = pipe && SDEPTH > 1;
    if constexpr (pipe) {
        if (np_ > 0) fetch(0, jn, sn_next);
        if constexpr (deep)
            if (np_ > PB) fetch(PB, jn2, sn_next2);
    }
    for (int s0 = 0; s0 < np_; s0 += PB) {
        int32_t jj[PB];
        Snap<T> pe[PB];
        if constexpr (deep) {
#pragma unroll
            for (int u = 0; u < PB; ++u) {
                jj[u] = jn[u]; pe[u] = sn_next[u];
                jn[u] = jn2[u]; sn_next[u] = sn_next2[u];
            }
            if (s0 + 2 * PB < np_) fetch(s0 + 2 * PB, jn2, sn_next2);
        } else if constexpr (pipe) {
#pragma unroll
            for (int u = 0; u < PB; ++u) { jj[u] = jn[u]; pe[u] = sn_next[u]; }
            if (s0 + PB < np_) fetch(s0 + PB, jn, sn_next);
        } else {
            fetch(s0, jj, pe);
        }
#pragma unroll
        for (int u = 0; u < PB; ++u) {
            if (s0 + u >= np_) break;
            const int32_t j = jj[u];
            const V3<T> cj = {pe[u].x, pe[u].y, pe[u].z};
            const T rj = pe[u].r;
            if constexpr (BOXES) {
                const int32_t kj = p.cs.kind[j];
                if (kind != 0 || kj != 0) {
                    // box-involved pair (rb_boxes.hpp), from step-start data of both
                    // bodies, in MuJoCo's geom order: sphere before box, boxes by id
                    auto emit = [&](const Contact<T> &con, int ck, bool self_g1) {
                        record(p, l, nrec, j, ck, con.dist);
                        const V3<T> n = (p.oriented && self_g1) ? V3<T>{-con.frame.x, -con.frame.y, -con.frame.z}
                                                                : con.frame;
                        solve_contact(p, con, x, n, m, k, invI, v, w);
                    };
                    M3<T> Mj;
                    const V3<T> hj = {p.cs.sx()[j], p.cs.sy()[j], p.cs.sz()[j]};
                    if (kj != 0) {
                        const T *qj = p.quat_cur + 4 * (int64_t)j;
                        Mj = mj_body_mat(Q4<T>{qj[0], qj[1], qj[2], qj[3]});
                    }
                    // geom1: the sphere of a sphere-box pair, else the lower id
                    // (one call of each primitive, operands selected)
                    const bool g1 = (kind == 0 && kj != 0) || (kind != 0 && kj != 0 && i < j);
                    const V3<T> p1 = g1 ? x : cj, p2 = g1 ? cj : x;
                    const V3<T> h1 = g1 ? sz : hj, h2 = g1 ? hj : sz;
                    M3<T> M1, M2;
#pragma unroll
                    for (int k = 0; k < 9; ++k) { M1.a[k] = g1 ? M.a[k] : Mj.a[k]; M2.a[k] = g1 ? Mj.a[k] : M.a[k]; }
                    if (kind == 0 || kj == 0) {
                        Contact<T> con;
                        if (sphere_box(p1, g1 ? sz.x : rj, p2, M2, h2, con)) emit(con, CK_SPHERE_BOX, g1);
                    } else {
                        box_box(p1, M1, h1, p2, M2, h2, poly, ps,
                                [&](const Contact<T> &c, int ck) { emit(c, ck, g1); });
                    }
                    continue;
                }
            }
            Contact<T> con;
            V3<T> n;
            if (i < j) {                        // this body is geom1
                sphere_sphere(x, sz.x, cj, rj, con);
                n = p.oriented ? V3<T>{-con.frame.x, -con.frame.y, -con.frame.z} : con.frame;
            } else {
                sphere_sphere(cj, rj, x, sz.x, con);
                n = con.frame;
            }
            record(p, l, nrec, j, 16, con.dist);
            solve_contact(p, con, x, n, m, k, invI, v, w);
        }
    }
    if (p.rec_count) p.rec_count[l] = nrec;
    STAMP(4);

    // ---- K3: integrate (collision.py:90-100) ---------------------------------
    if (p.bounds) {                              // peer-to-peer exchange: the step-start cell too
        int32_t cx, cy, cz;
        if (cell_of(x.x, x.y, x.z, p.grid.inv_cs, cx, cy, cz)) { cell[3] = cx; cell[4] = cy; cell[5] = cz; }
    }
    x = {x.x + v.x * p.dt, x.y + v.y * p.dt, x.z + v.z * p.dt};
    Snap<T> sn;
    sn.x = x.x; sn.y = x.y; sn.z = x.z; sn.r = bi;
    // next step's broadphase: the slot atomic goes first (a later load or
    // atomic would wait for every older store), its round trip overlaps the
    // snapshot store and the quaternion update
    Claim cl{0u, 0, 0ull, 0u, 0};
    // the one-lane and wide forms (and the split form's update) run in
    // linear-layout worlds only; the cooperative form and the box kernel
    // read the layout
    constexpr int L = (PM == 2 || (PM == 0 && !BOXES)) ? LAYOUT_LINEAR : LAYOUT_ANY;
    // heads per line: known in the cooperative and wide forms (rb_capi.hip)
    constexpr int RL = PM == 1 ? 0 : PM == 2 ? 2 : -1;
    if (p.next.line) cl = claim_slot<L, RL>(p.grid, p.next, p.err, sn, gen_next);
    wt_store(p.snap_next + i, sn);
    if (p.bounds) {                              // peer-to-peer exchange: this body's new cell
        int32_t cx, cy, cz;
        if (cell_of(sn.x, sn.y, sn.z, p.grid.inv_cs, cx, cy, cz)) { cell[0] = cx; cell[1] = cy; cell[2] = cz; }
    }
    STAMP(5);
    const Q4<T> res = mj_mulquat(Q4<T>{T(0), w.x, w.y, w.z}, q);
    Q4<T> qn = {q.w + (T(0.5) * res.w) * p.dt, q.x + (T(0.5) * res.x) * p.dt,
                q.y + (T(0.5) * res.y) * p.dt, q.z + (T(0.5) * res.z) * p.dt};
    const T nq = sqroot(fmadd(qn.z, qn.z, fmadd(qn.y, qn.y, fmadd(qn.x, qn.x, qn.w * qn.w))));
    qn = {qn.w / nq, qn.x / nq, qn.y / nq, qn.z / nq};
    wt_store(p.st.vx() + l, v.x); wt_store(p.st.vy() + l, v.y); wt_store(p.st.vz() + l, v.z);
    wt_store(p.st.wx() + l, w.x); wt_store(p.st.wy() + l, w.y); wt_store(p.st.wz() + l, w.z);
    wt_store(p.st.qw() + l, qn.w); wt_store(p.st.qx() + l, qn.x); wt_store(p.st.qy() + l, qn.y);
    wt_store(p.st.qz() + l, qn.z);
    // next step's orientation snapshot (box worlds), from every kernel that
    // steps a box: the box kernel reads it for a partner that was out of any
    // box pair's range (stepped by a sphere kernel) in the step before
    if (p.quat_next && kind != 0) {
        T *qs = p.quat_next + 4 * (int64_t)i;
        wt_store(qs + 0, qn.w); wt_store(qs + 1, qn.x); wt_store(qs + 2, qn.y); wt_store(qs + 3, qn.z);
    }
    publish_slot<RL>(p.next, p.err, cl, sn, (uint32_t)i | (kind != 0 ? BOX_FLAG : 0u));
    STAMP(6);
}

// One body (G lanes): contact search, then (lane 0) the update.  WIDE: the
// one-lane form for one wave per SIMD (search_buckets_wide; state loads and
// inv(I_w) under the head loads).
template <typename T, int MAXP, int G, bool WIDE, bool BOXES, bool PRE = false, bool HELP = false>
__device__ __forceinline__ void body_step(const StepParams<T> &p, const Lead<T> &ld, bool active, int64_t lb, int slot,
                                          int k, int tid,
                                          int32_t *s_id, Snap<T> *s_pos, int32_t *t_id, Snap<T> *t_pos,
                                          uint32_t *s_cand, int32_t *cell, uint32_t gen, T *s_poly,
                                          uint8_t *s_didx = nullptr, Snap<T> *s_hpos = nullptr,
                                          const T *s_help = nullptr) {
    constexpr int NB = STEP_BLOCK / G;
    const int32_t l = active ? (int32_t)lb : 0;
    const int32_t i = ld.lo + l;

    // ---- K1 first: the contact search reads only step-start data -----------
    const Snap<T> self = xld(ld.snap_cur + i);
    const V3<T> x = {self.x, self.y, self.z};
    const int32_t ci = RB_ABLATE == 8 ? 0 : i;    // (diagnostic, load_body)
    const int32_t kind = ld.cs.kind[ci];
    const T bi = self.r;
    // half extents y, z only matter for boxes; loaded for every body (a load
    // under a kind test would wait for kind before the state loads issue)
    const T sy = ld.cs.sy()[ci], szz = ld.cs.sz()[ci];
    const V3<T> sz = {ld.cs.sx()[ci], kind != 0 ? sy : T(0), kind != 0 ? szz : T(0)};
    BodyIn<T> in;
    LazyInvI<T> invI;
    bool forced = false;
    // state loads issued before the search (the wide form measured 5 % slower
    // with them issued after the bucket heads, C3)
    constexpr bool early = G > 1 || WIDE;
    if constexpr (early && HELP && WIDE) {
        // the helper wave loads the state and constants (help_body) and hands
        // over q, m, inv(I_w) and the post-gravity, post-plane v and w: the
        // body lanes load only what the search needs (the cooperative form
        // keeps its own loads: handing q, m over there measured 4,096 bodies
        // 7.4 -> 7.9 us, 8,190 8.6 -> 9.0)
    } else if constexpr (early) {
        in = load_body(ld.st, ld.cs, l, i);
        invI.I = in.I;
        invI.q = in.q;
    }
    if constexpr (PRE) {
        // preloaded lead (step_body): the parameter block's fields the search
        // starts with, in one scalar round trip under the body's loads (which
        // needed none of them)
        asm volatile("" ::"s"(p.grid.inv_cs), "s"(p.grid.H), "s"(p.grid.super), "s"(p.cur.line), "s"(p.cur.gen),
                     "s"(p.n_global), "s"(p.xfrc));
        if constexpr (G > 1) asm volatile("" ::"s"(p.cur.pos));
        gen = *p.cur.gen;
    }
    STAMP(1);
    int32_t np_ = 0;
    bool defer = false;                          // a box-involved partner in range: the box kernel steps it
    if constexpr (G == 1 && WIDE && HELP) {
        // the helper wave evaluates inv(I_w), gravity and the plane contacts
        // (help_body); every lane of the body wave takes part in its two
        // barriers, so the search runs under the active mask only
        if (RB_ABLATE != 1 && active)
            np_ = search_partners_wide<T, MAXP, BOXES>(p, i, kind, x, sz.x, bi, s_id, s_cand, s_didx, s_hpos, tid, gen,
                                                       defer, [] {});
        __syncthreads();                         // the search is done with s_cand: the helper fills it
        __syncthreads();
    } else if constexpr (G == 1 && WIDE) {
        if (RB_ABLATE != 1)
            np_ = search_partners_wide<T, MAXP, BOXES>(p, i, kind, x, sz.x, bi, s_id, s_cand, s_didx, s_hpos, tid, gen,
                                                       defer, [&] {
                invI.get();
                if (!p.xfrc) {
                    apply_force(p, l, in.m, invI, in.v, in.w);
                    forced = true;
                }
            });
    } else if constexpr (G == 1) {
        if (RB_ABLATE != 1) np_ = search_partners<T, MAXP, BOXES>(p, i, kind, x, sz.x, bi, s_id, tid, gen, defer);
    } else if constexpr (HELP) {
        // the helper wave evaluates inv(I_w) and gravity (help_body)
        if (RB_ABLATE != 1)
            np_ = search_coop<T, MAXP, G, BOXES, 0>(p, active, i, kind, x, sz.x, bi, s_id, s_pos, t_id, t_pos, slot, k, tid,
                                                    gen, defer, [] {});
    } else {
        if (RB_ABLATE != 1)
            np_ = search_coop<T, MAXP, G, BOXES, 0>(p, active, i, kind, x, sz.x, bi, s_id, s_pos, t_id, t_pos, slot, k, tid,
                                          gen, defer, [&] {
                                              invI.get();
                                              if (!p.xfrc) {
                                                  apply_force(p, l, in.m, invI, in.v, in.w);
                                                  forced = true;
                                              }
                                          });
    }
    STAMP(2);
    if (RB_ABLATE == 7) np_ = 0;                 // diagnostic: search, but solve no partner contact
    if (!active || k != 0 || RB_ABLATE == 4) return;
    if (!BOXES && defer) {                       // box worlds only (p.defer_q set)
        // queued for the box kernel; chunks replayed without it (rb_capi.hip
        // box_opt) only count, and are rolled back if the count is not zero
        const int32_t q = atomicAdd(p.defer_cnt, 1);
        if (q < p.S) p.defer_q[q] = l;
        return;
    }
    if constexpr (!early) {
        in = load_body(p, l, i);
        invI.I = in.I;
        invI.q = in.q;
    }
    bool help_planes = false;
    int32_t help_nrec = 0;
    if constexpr (HELP) {
        // the helper's results (its LDS writes precede the search's barriers)
        const T *o = s_help + slot;
        constexpr int NBH = STEP_BLOCK / G;
#pragma unroll
        for (int e = 0; e < 9; ++e) invI.m.a[e] = o[e * NBH];
        invI.have = true;
        if (!p.xfrc) {
            in.v = {o[9 * NBH], o[10 * NBH], o[11 * NBH]};
            in.w = {o[12 * NBH], o[13 * NBH], o[14 * NBH]};
            forced = true;
        } else if constexpr (WIDE) {             // applied forces: the body lanes apply them
            in.v = {p.st.vx()[l], p.st.vy()[l], p.st.vz()[l]};
            in.w = {p.st.wx()[l], p.st.wy()[l], p.st.wz()[l]};
        }
        if constexpr (WIDE) {
            in.q = {o[16 * NBH], o[17 * NBH], o[18 * NBH], o[19 * NBH]};
            in.m = o[20 * NBH];
        }
        const T pr = o[15 * NBH];
        help_planes = pr >= T(0);
        help_nrec = help_planes ? (int32_t)pr : 0;
    }
    constexpr int PM = G > 1 ? 1 : (WIDE && RB_WIDE_LDSPOS) ? 2 : 0;
    constexpr int SD = (WIDE && HELP) ? RB_SOLVE_DEPTH : 1;
    body_update<T, PM, BOXES, SD>(p, l, i, x, kind, sz, bi, in, forced, invI, np_, s_id + slot, NB,
                                  PM == 2 ? s_hpos + slot : s_pos + slot, tid, cell, gen + 1u,
                                  BOXES ? s_poly + slot : nullptr, NB, PM == 2 ? s_didx + slot : nullptr, help_nrec,
                                  help_planes);
}

// Halo exchange: fold the wave's new cells, given as per-lane boxes
// (lo[0] == INT32_MAX: none), into the step's bound copies — one atomic
// min/max per axis per wave, on copy (block % BOUND_COPIES).  Every lane of
// the wave must call it.
__device__ __forceinline__ void fold_box(int32_t *bounds, int32_t lo[3], int32_t hi[3]) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            lo[d] = min(lo[d], __shfl_xor(lo[d], off));
            hi[d] = max(hi[d], __shfl_xor(hi[d], off));
        }
    if ((threadIdx.x & 63) == 0 && lo[0] != INT32_MAX) {
        int32_t *c = bounds + (int64_t)(blockIdx.x % BOUND_COPIES) * BOUND_STRIDE;
#pragma unroll
        for (int d = 0; d < 3; ++d) { atomicMin(c + d, lo[d]); atomicMax(c + 3 + d, hi[d]); }
    }
}
// one cell per lane (cell[0] == INT32_MAX: none)
__device__ __forceinline__ void fold_bounds(int32_t *bounds, const int32_t *cell) {
    int32_t lo[3], hi[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const bool have = cell[0] != INT32_MAX;
        lo[d] = have ? cell[d] : INT32_MAX;
        hi[d] = have ? cell[d] : INT32_MIN;
    }
    fold_box(bounds, lo, hi);
}

// Helper wave of the cooperative form (HELP): one lane per body of the
// workgroup evaluates inv(I_w), gravity and a sphere's plane contacts (the
// first in its contact order) — VALU chain the body lanes otherwise run
// under or after their bucket loads — and leaves inv(I_w), v, w and the
// recorded-contact count, q and m in LDS (column layout, HELP_REALS per body) before
// the search's first barrier; it then takes part in the search's two
// barriers.  The same arithmetic in the same order, so bit-identical.
//
// WIDE (step_kernel_wide_help): the results go to the body wave's candidate
// list area once its search is done with it (between the two barriers),
// so the workgroup's LDS stays within a quarter of the CU's.
constexpr int HELP_REALS = 21;                   // inv(I_w) 9, v 3, w 3, records 1, q 4, m 1
template <typename T, int NB, bool WIDE = false>
__device__ __forceinline__ void help_body(const StepParams<T> &p, const Lead<T> &ld, int h, T *s_help) {
    // the same block -> bodies mapping as the body lanes (step_body)
    const int64_t hb = (int64_t)xcd_block(blockIdx.x, gridDim.x) * NB + h;
    const bool act = h < NB && hb < ld.n_local;
    // results kept in registers across the wide form's first barrier; the
    // barriers themselves are outside every divergent branch (a barrier in
    // a branch taken by some lanes of the wave would be issued once per path)
    BodyIn<T> in{};
    M3<T> m{};
    int32_t nrec = 0;
    bool planes = false;
    if (act) {
        const int32_t l = (int32_t)hb, i = ld.lo + l;
        in = load_body(ld.st, ld.cs, l, i);
        LazyInvI<T> invI;
        invI.I = in.I;
        invI.q = in.q;
        m = invI.get();
        if (!p.xfrc) {
            apply_force(p, l, in.m, invI, in.v, in.w);
            // a body's plane contacts come first in its contact order
            // (body_update: a sphere's one per plane, a box's corners), so
            // they are solved here too
            const int32_t kind = ld.cs.kind[i];
            const Snap<T> self = ld.snap_cur[i];
            const V3<T> x = {self.x, self.y, self.z};
            const T k = impulse_k(in.m);
            if (kind == 0) {
                const T rad = ld.cs.sx()[i];
                for (int pl = 0; pl < p.n_planes; ++pl) {
                    const V3<T> pn = {p.pn[pl][0], p.pn[pl][1], p.pn[pl][2]};
                    const V3<T> pp = {p.pp[pl][0], p.pp[pl][1], p.pp[pl][2]};
                    Contact<T> con;
                    if (!plane_sphere(pn, pp, x, rad, con)) continue;
                    record(p, l, nrec, -1 - pl, 0, con.dist);
                    solve_contact(p, con, x, con.frame, in.m, k, invI, in.v, in.w);
                }
            } else {
                const V3<T> sz = {ld.cs.sx()[i], ld.cs.sy()[i], ld.cs.sz()[i]};
                const M3<T> M = mj_body_mat(in.q);
                for (int pl = 0; pl < p.n_planes; ++pl) {
                    const V3<T> pn = {p.pn[pl][0], p.pn[pl][1], p.pn[pl][2]};
                    const V3<T> dif = {x.x - p.pp[pl][0], x.y - p.pp[pl][1], x.z - p.pp[pl][2]};
                    const T dist = mj_dot(dif, pn);
                    int cnt = 0;
                    for (int c = 0; c < 8 && cnt < 4; ++c) {
                        Contact<T> con;
                        if (!plane_box_corner(pn, x, dist, M, sz, c, con)) continue;
                        ++cnt;
                        record(p, l, nrec, -1 - pl, 1 + c, con.dist);
                        solve_contact(p, con, x, con.frame, in.m, k, invI, in.v, in.w);
                    }
                }
            }
            planes = true;
        }
    }
    if (WIDE) __syncthreads();                   // the body wave's search is done with s_cand
    if (act) {
        T *o = s_help + h;
#pragma unroll
        for (int e = 0; e < 9; ++e) o[e * NB] = m.a[e];
        o[9 * NB] = in.v.x; o[10 * NB] = in.v.y; o[11 * NB] = in.v.z;
        o[12 * NB] = in.w.x; o[13 * NB] = in.w.y; o[14 * NB] = in.w.z;
        o[15 * NB] = T(planes ? nrec : -1);
        o[16 * NB] = in.q.w; o[17 * NB] = in.q.x; o[18 * NB] = in.q.y; o[19 * NB] = in.q.z;
        o[20 * NB] = in.m;
    }
    __syncthreads();
    if (!WIDE) __syncthreads();                  // search_coop's two barriers
}

// HALO: the halo push compiled in (checked at run time: p.halo.mail); the
// wide forms — the single-GPU bench's kernels — are also instantiated
// without it (launch_step_wide picks), which measured 1-2 % faster at C3
template <typename T, int MAXP, int G, bool WIDE = false, bool BOXES = false, bool HELP = false, bool HALO = true>
__device__ __forceinline__ void step_body(const StepParams<T> &p, const Lead<T> &ld) {
    constexpr int NB = STEP_BLOCK / G;          // bodies per workgroup
    __shared__ int32_t s_id[MAXP * NB];
    __shared__ T s_poly[BOXES ? 48 * NB : 1];   // box-box face clipping: 2 x 8 vertices x 3 per body
    __shared__ uint32_t s_cand[WIDE ? WIDE_MAXC * NB : 1];
    __shared__ uint8_t s_didx[WIDE ? MAXP * NB : 1];
    __shared__ Snap<T> s_hpos[WIDE && RB_WIDE_LDSPOS ? WIDE_HPOS * NB : 1];
    __shared__ int32_t t_id[G > 1 ? MAXP * NB : 1];
    __shared__ Snap<T> s_pos[G > 1 ? MAXP * NB : 1];
    __shared__ Snap<T> t_pos[G > 1 ? MAXP * NB : 1];
    // the wide form's helper results share the candidate list's area
    __shared__ T s_help[HELP && !WIDE ? HELP_REALS * NB : 1];
    static_assert(!WIDE || sizeof(uint32_t) * WIDE_MAXC >= HELP_REALS * sizeof(T), "helper results fit in s_cand");
    T *const help_lds = WIDE ? reinterpret_cast<T *>(s_cand) : s_help;
    const int tid = threadIdx.x;
    if (RB_ABLATE == 3) return;
    if constexpr (HELP) {
        static_assert(!BOXES, "helper waves: the sphere step kernels");
        if (tid >= STEP_BLOCK) {                 // the workgroup's second wave
            help_body<T, NB, WIDE>(p, ld, tid - STEP_BLOCK, help_lds);
            return;
        }
    }
    STAMP(0);
#if RB_STAMPS
    // placement: HW_ID (wave, SIMD, CU, SE fields) and XCC_ID of the block's first wave
    if (tid == 0 && blockIdx.x < (1u << 16)) {
        rb_stamp_buf[blockIdx.x][15] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        rb_stamp_buf[blockIdx.x][14] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    }
#endif
    // The lead (the body's first loads' fields) is preloaded; body_step waits
    // for the parameter block's scalar loads only under the body's loads.
    // Block 0 advances the exchange's step number and publishes the next
    // table's generation (one more than the one this step reads) for the
    // kernels that insert after this one, at the end: a store ahead of the
    // body loads would hold them back (they may not pass it).

    const int slot = tid / G, k = tid % G;
    const int64_t lb = (int64_t)xcd_block(blockIdx.x, gridDim.x) * NB + slot;
    const int64_t halo_e = HALO && p.halo.mail ? *p.halo.halo_e : 0;   // (halo-exchanging shards: the push's epoch)
    const bool active = lb < ld.n_local;
    int32_t cell[6] = {INT32_MAX, 0, 0, 0, 0, 0};   // new cell, step-start cell (peer-to-peer exchange)
    if (G > 1 || HELP || active)                 // (a helper's barriers: every lane)
        body_step<T, MAXP, G, WIDE, BOXES, true, HELP>(p, ld, active, lb, slot, k, tid, s_id, s_pos, t_id, t_pos, s_cand,
                                                       cell, 0u /* loaded in body_step */, s_poly, s_didx, s_hpos, help_lds);
    if (p.bounds) fold_bounds(p.bounds, cell);
    if (HALO && p.halo.mail) {                   // halo-exchanging shard: push to the peers
        int32_t b[6];
        if (halo_bounds(p, halo_e, b)) halo_push(p, halo_e, cell[0] != INT32_MAX, (int32_t)(ld.lo + lb), cell, b);
    }
    if (blockIdx.x == 0 && tid == 0) {
        if (p.next.line) *p.next.gen = *p.cur.gen + 1u;
        if (p.epoch) *p.epoch += 1;
    }
}

// The two forms as separate kernels: the one-lane (large-scene) form may be
// compiled for more waves per SIMD — its dependent random loads want
// occupancy more than registers — without touching the cooperative form.
#ifndef RB_MIN_WAVES_G1
#define RB_MIN_WAVES_G1 1
#endif
// the cooperative form fits 3 waves per SIMD without spilling (measured:
// +9-12% at 32k-65k bodies, unchanged at 4k; 4 waves spill and lose)
#ifndef RB_MIN_WAVES_COOP
#define RB_MIN_WAVES_COOP 3
#endif
template <typename T, int MAXP>
__global__ __launch_bounds__(STEP_BLOCK)
__attribute__((amdgpu_waves_per_eu(MAXP <= 16 ? RB_MIN_WAVES_COOP : 2)))   // 32 partners: 2 fit
void step_kernel_coop(const Snap<T> *snap_cur, T *st_base, int64_t st_S, const T *cs_base, int64_t cs_Npad,
                      const int32_t *cs_kind, int32_t n_local, int32_t lo, StepParams<T> p) {
    step_body<T, MAXP, 8, false, false>(
        p, Lead<T>{snap_cur, BodyState<T>{st_base, st_S}, BodyConsts<T>{cs_base, cs_Npad, cs_kind}, n_local, lo});
}
// the cooperative form with a helper wave per workgroup (help_body): small
// scenes, whose body waves leave SIMDs idle
template <typename T, int MAXP>
__global__ __launch_bounds__(2 * STEP_BLOCK)
__attribute__((amdgpu_waves_per_eu(MAXP <= 16 ? RB_MIN_WAVES_COOP : 2)))
void step_kernel_coop_help(const Snap<T> *snap_cur, T *st_base, int64_t st_S, const T *cs_base, int64_t cs_Npad,
                           const int32_t *cs_kind, int32_t n_local, int32_t lo, StepParams<T> p) {
    step_body<T, MAXP, 8, false, false, true>(
        p, Lead<T>{snap_cur, BodyState<T>{st_base, st_S}, BodyConsts<T>{cs_base, cs_Npad, cs_kind}, n_local, lo});
}
template <typename T, int MAXP>
__global__ __launch_bounds__(STEP_BLOCK)
#if RB_MIN_WAVES_G1 > 1
__attribute__((amdgpu_waves_per_eu(RB_MIN_WAVES_G1)))
#endif
void step_kernel_one(const Snap<T> *snap_cur, T *st_base, int64_t st_S, const T *cs_base, int64_t cs_Npad,
                     const int32_t *cs_kind, int32_t n_local, int32_t lo, StepParams<T> p) {
    step_body<T, MAXP, 1, false, false>(
        p, Lead<T>{snap_cur, BodyState<T>{st_base, st_S}, BodyConsts<T>{cs_base, cs_Npad, cs_kind}, n_local, lo});
}
// The box kernel (box worlds, after the step kernel): steps the bodies the
// step kernel deferred — those with a box-involved partner within bounding
// range — one lane per body with the box narrowphase (rb_boxes.hpp), from
// the same step-start data, so the step stays Jacobi across bodies.  One
// wave per SIMD: the narrowphase's registers fit without scratch, and the
// sphere step kernels keep their occupancy.
template <typename T, int MAXP>
__global__ __launch_bounds__(STEP_BLOCK) __attribute__((amdgpu_waves_per_eu(1, 1)))
void box_kernel(StepParams<T> p) {
    __shared__ int32_t s_id[MAXP * STEP_BLOCK];
    __shared__ T s_poly[48 * STEP_BLOCK];
    const int tid = threadIdx.x;
    const uint32_t gen = *p.cur.gen;
    const int32_t n = *p.defer_cnt;
    int32_t lo[3] = {INT32_MAX, INT32_MAX, INT32_MAX}, hi[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
    // halo-exchanging shard: the peers' bounds, read with every lane active
    int32_t hb[6];
    const int64_t halo_e = p.halo.mail ? *p.halo.halo_e : 0;
    const bool halo = p.halo.mail && n > (int32_t)(blockIdx.x * STEP_BLOCK) && halo_bounds(p, halo_e, hb);
    for (int64_t qi0 = (int64_t)blockIdx.x * STEP_BLOCK; qi0 < n; qi0 += (int64_t)gridDim.x * STEP_BLOCK) {
        const int64_t qi = qi0 + tid;
        int32_t cell[6] = {INT32_MAX, 0, 0, 0, 0, 0};
        int32_t l = 0;
        // one lane per body: the lane's LDS column (partner list, polygon) is slot = tid
        if (qi < n) {
            l = p.defer_q[qi];
            body_step<T, MAXP, 1, false, true>(p, Lead<T>::of(p), true, l, tid, 0, tid, s_id, nullptr, nullptr, nullptr,
                                               nullptr, cell, gen, s_poly);
        }
        if (halo) halo_push(p, halo_e, cell[0] != INT32_MAX, p.lo + l, cell, hb);   // (every lane of the wave)
        if (cell[0] != INT32_MAX)
#pragma unroll
            for (int d = 0; d < 3; ++d) { lo[d] = min(lo[d], cell[d]); hi[d] = max(hi[d], cell[d]); }
    }
    // halo exchange: the deferred bodies' new cells (the step kernel folded
    // only the bodies it stepped itself)
    if (p.bounds) fold_box(p.bounds, lo, hi);
    if (blockIdx.x == 0 && tid == 0) *p.defer_reset = 0;    // the next step's queue
}
// one wave per SIMD (up to 64 x 1024 owned bodies): every register is free
template <typename T, int MAXP, bool HALO>
__global__ __launch_bounds__(STEP_BLOCK) __attribute__((amdgpu_waves_per_eu(1, 1)))
void step_kernel_wide(const Snap<T> *snap_cur, T *st_base, int64_t st_S, const T *cs_base, int64_t cs_Npad,
                      const int32_t *cs_kind, int32_t n_local, int32_t lo, StepParams<T> p) {
    step_body<T, MAXP, 1, true, false, false, HALO>(
        p, Lead<T>{snap_cur, BodyState<T>{st_base, st_S}, BodyConsts<T>{cs_base, cs_Npad, cs_kind}, n_local, lo});
}

// the wide form with a helper wave per workgroup (help_body): two waves per
// SIMD, each within 256 registers
template <typename T, int MAXP, bool HALO>
__global__ __launch_bounds__(2 * STEP_BLOCK) __attribute__((amdgpu_waves_per_eu(2, 2)))
void step_kernel_wide_help(const Snap<T> *snap_cur, T *st_base, int64_t st_S, const T *cs_base, int64_t cs_Npad,
                           const int32_t *cs_kind, int32_t n_local, int32_t lo, StepParams<T> p) {
    step_body<T, MAXP, 1, true, false, true, HALO>(
        p, Lead<T>{snap_cur, BodyState<T>{st_base, st_S}, BodyConsts<T>{cs_base, cs_Npad, cs_kind}, n_local, lo});
}

// ---- split form (large scenes): search kernel + update kernel -------------
// The fused kernel's register footprint (the f64 solve) caps it at two
// waves per SIMD, too few to hide the search's dependent random loads.
// Split, the search runs at high occupancy and hands each body's sorted
// partner ids to the update through a per-slot list in HBM ([MAXP][S],
// coalesced by slot).
template <typename T, int MAXP, int G>
__global__ __launch_bounds__(STEP_BLOCK) void search_kernel(StepParams<T> p) {
    constexpr int NB = STEP_BLOCK / G;
    __shared__ int32_t s_id[MAXP * NB];
    __shared__ int32_t t_id[G > 1 ? MAXP * NB : 1];
    __shared__ Snap<T> s_pos[G > 1 ? MAXP * NB : 1];
    __shared__ Snap<T> t_pos[G > 1 ? MAXP * NB : 1];
    const int tid = threadIdx.x;
    const int slot = tid / G, k = tid % G;
    const int64_t lb = (int64_t)blockIdx.x * NB + slot;
    const bool active = lb < p.n_local;
    if (G == 1 && !active) return;
    const int32_t l = active ? (int32_t)lb : 0;
    const int32_t i = p.lo + l;
    const Snap<T> self = p.snap_cur[CHK(i, p.n_global)];
    const V3<T> x = {self.x, self.y, self.z};
    const int32_t kind = p.cs.kind[i];
    const T rad = p.cs.sx()[i];
    const uint32_t gen = *p.cur.gen;
    int32_t np_;
    bool defer = false;                          // split form: sphere worlds only
    if constexpr (G == 1) np_ = search_partners<T, MAXP, false>(p, i, kind, x, rad, self.r, s_id, tid, gen, defer);
    else np_ = search_coop<T, MAXP, G, false, -1>(p, active, i, kind, x, rad, self.r, s_id, s_pos, t_id, t_pos, slot, k, tid,
                                       gen, defer, [] {});
    if (!active) return;
    for (int s = k; s < np_; s += G) p.plist[CHK((int64_t)s * p.S + l, (int64_t)MAXP * p.S)] = s_id[s * NB + slot];
    if (k == 0) p.plist_cnt[CHK(l, p.S)] = np_;
}

template <typename T>
__global__ __launch_bounds__(STEP_BLOCK) void update_kernel(StepParams<T> p) {
    const int tid = threadIdx.x;
    const int64_t gt = (int64_t)blockIdx.x * STEP_BLOCK + tid;
    const int64_t lb = gt;
    int32_t cell[6] = {INT32_MAX, 0, 0, 0, 0, 0};
    const uint32_t gen_next = *p.cur.gen + 1u;
    const int64_t halo_e = p.halo.mail ? *p.halo.halo_e : 0;
    if (p.next.line && blockIdx.x == 0 && tid == 0) *p.next.gen = gen_next;
    if (lb < p.n_local) {
        const int32_t l = (int32_t)lb, i = p.lo + l;
        const Snap<T> self = p.snap_cur[CHK(i, p.n_global)];
        const V3<T> x = {self.x, self.y, self.z};
        const int32_t kind = p.cs.kind[i];
        const V3<T> sz = {p.cs.sx()[i], kind != 0 ? p.cs.sy()[i] : T(0), kind != 0 ? p.cs.sz()[i] : T(0)};
        const BodyIn<T> in = load_body(p, l, i);
        LazyInvI<T> invI;
        invI.I = in.I;
        invI.q = in.q;
        const int32_t np_ = p.plist_cnt[CHK(l, p.S)];
        if (RB_BOUNDS && np_ > 16) printf("RB_BOUNDS np_ %d at l %d\n", np_, l);
        body_update<T, 0>(p, l, i, x, kind, sz, self.r, in, false, invI, np_, p.plist + l, p.S, nullptr, tid,
                          cell, gen_next);
    }
    if (p.bounds) fold_bounds(p.bounds, cell);
    if (p.halo.mail) {                           // halo-exchanging shard: push to the peers
        int32_t b[6];
        if (halo_bounds(p, halo_e, b)) halo_push(p, halo_e, cell[0] != INT32_MAX, (int32_t)(p.lo + lb), cell, b);
    }
}

#if RB_STAMPS
extern "C" int rb_diag_stamps(unsigned long long *out, int nblocks) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(rb_stamp_buf), sizeof(unsigned long long) * 16 * nblocks);
}
#endif

// ---- known-answer kernels ----------------------------------------------
template <typename T>
__global__ void kat_impulse_kernel(int64_t n, const double *in, double *out) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const double *a = in + 24 * c;
    const T m = (T)a[0], e = (T)a[1], mu = (T)a[2];
    V3<T> v = {(T)a[3], (T)a[4], (T)a[5]}, w = {(T)a[6], (T)a[7], (T)a[8]};
    const V3<T> r = {(T)a[9], (T)a[10], (T)a[11]}, nn = {(T)a[12], (T)a[13], (T)a[14]};
    M3<T> Iw;
    for (int k = 0; k < 9; ++k) Iw.a[k] = (T)a[15 + k];
    const M3<T> invI = np_inv3(Iw);
    T jn;
    V3<T> jt;
    impulse(impulse_k(m), v, w, r, nn, e, mu, jn, jt);
    apply(v, w, m, invI, r, nn, jn, jt);      // the reference always applies
    double *o = out + 10 * c;
    o[0] = jn; o[1] = jt.x; o[2] = jt.y; o[3] = jt.z;
    o[4] = v.x; o[5] = v.y; o[6] = v.z; o[7] = w.x; o[8] = w.y; o[9] = w.z;
}

template <typename T>
__global__ void kat_inertia_kernel(int64_t n, const double *in, double *out) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const double *a = in + 7 * c;
    const M3<T> Iw = inertia_world(V3<T>{(T)a[0], (T)a[1], (T)a[2]}, Q4<T>{(T)a[3], (T)a[4], (T)a[5], (T)a[6]});
    const M3<T> Ii = np_inv3(Iw);
    for (int k = 0; k < 9; ++k) { out[18 * c + k] = Iw.a[k]; out[18 * c + 9 + k] = Ii.a[k]; }
}

template <typename T>
__global__ void kat_apply_kernel(int64_t n, const double *in, double *out) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const double *a = in + 26 * c;
    const T m = (T)a[0];
    V3<T> v = {(T)a[1], (T)a[2], (T)a[3]}, w = {(T)a[4], (T)a[5], (T)a[6]};
    const V3<T> r = {(T)a[7], (T)a[8], (T)a[9]}, nn = {(T)a[10], (T)a[11], (T)a[12]};
    const T jn = (T)a[13];
    const V3<T> jt = {(T)a[14], (T)a[15], (T)a[16]};
    M3<T> Iw;
    for (int k = 0; k < 9; ++k) Iw.a[k] = (T)a[17 + k];
    apply(v, w, m, np_inv3(Iw), r, nn, jn, jt);
    double *o = out + 6 * c;
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = w.x; o[4] = w.y; o[5] = w.z;
}

// in[22] = kind1, kind2, c1[3], q1[4], s1[3], c2[3], q2[4], s2[3] (body 1 =
// lower id) -> out[33] = count, then per contact dist, pos[3], frame[3], kind
template <typename T>
__global__ __launch_bounds__(64) void kat_narrow_kernel(int64_t n, const double *in, double *out) {
    __shared__ T s_poly[48 * 64];
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const double *a = in + 22 * c;
    double *o = out + 33 * c;
    for (int k = 0; k < 33; ++k) o[k] = 0;
    const int k1 = (int)a[0], k2 = (int)a[1];
    const V3<T> c1 = {(T)a[2], (T)a[3], (T)a[4]}, c2 = {(T)a[12], (T)a[13], (T)a[14]};
    const Q4<T> q1 = {(T)a[5], (T)a[6], (T)a[7], (T)a[8]}, q2 = {(T)a[15], (T)a[16], (T)a[17], (T)a[18]};
    const V3<T> s1 = {(T)a[9], (T)a[10], (T)a[11]}, s2 = {(T)a[19], (T)a[20], (T)a[21]};
    int m = 0;
    auto emit = [&](const Contact<T> &con, int ck) {
        double *r = o + 1 + 8 * m;
        r[0] = (double)con.dist;
        r[1] = (double)con.pos.x; r[2] = (double)con.pos.y; r[3] = (double)con.pos.z;
        r[4] = (double)con.frame.x; r[5] = (double)con.frame.y; r[6] = (double)con.frame.z;
        r[7] = ck;
        ++m;
    };
    Contact<T> con;
    if (k1 == 0 && k2 == 0) {
        if (sphere_sphere(c1, s1.x, c2, s2.x, con)) emit(con, 16);
    } else if (k1 == 0) {
        if (sphere_box(c1, s1.x, c2, mj_body_mat(q2), s2, con)) emit(con, CK_SPHERE_BOX);
    } else if (k2 == 0) {
        if (sphere_box(c2, s2.x, c1, mj_body_mat(q1), s1, con)) emit(con, CK_SPHERE_BOX);
    } else {
        box_box(c1, mj_body_mat(q1), s1, c2, mj_body_mat(q2), s2, s_poly + threadIdx.x, 64, emit);
    }
    o[0] = m;
}

// ---- launchers ----------------------------------------------------------
// The wide form's kernels live in their own unit (RB_WIDE_UNIT=1, built with
// the memory-clause scheduling flags): the other units must call that unit's
// instantiation, not compile (and, through the linker's choice among weak
// copies, possibly run) a copy of their own
#if defined(RB_WIDE_UNIT) && RB_WIDE_UNIT == 0
extern template hipError_t launch_step_wide<double>(const StepParams<double> &, int, bool, hipStream_t);
extern template hipError_t launch_step_wide<float>(const StepParams<float> &, int, bool, hipStream_t);
#endif
template <typename T> hipError_t launch_step(const StepParams<T> &p, int maxp, int form, bool boxes, hipStream_t s) {
    const bool coop = form == FORM_COOP || form == FORM_COOP_HELP;
    const int nb = coop ? STEP_BLOCK / 8 : STEP_BLOCK;
    int64_t blocks = (p.n_local + nb - 1) / nb;
    if (blocks < 1) blocks = 1;
    const bool split = !coop && p.plist && !boxes;
    if (boxes && (!p.quat_cur || !p.defer_q || !p.defer_cnt || !p.defer_reset)) return hipErrorInvalidValue;
    // the cooperative search reads bucket slot snapshots: never launch it
    // on a table without them
    if (needs_slot_snapshots(coop, split) && (!p.cur.pos || (p.next.line && !p.next.pos))) return hipErrorInvalidValue;
    if (split) {
        constexpr int GS = SPLIT_SEARCH_LANES;
        const int64_t sblocks = blocks * GS;
        if (maxp <= 16) hipLaunchKernelGGL((search_kernel<T, 16, GS>), dim3((unsigned)sblocks), dim3(STEP_BLOCK), 0, s, p);
        else hipLaunchKernelGGL((search_kernel<T, 32, GS>), dim3((unsigned)sblocks), dim3(STEP_BLOCK), 0, s, p);
        hipLaunchKernelGGL((update_kernel<T>), dim3((unsigned)blocks), dim3(STEP_BLOCK), 0, s, p);
    } else if (coop && form == FORM_COOP_HELP) {   // (box worlds: the box kernel follows)
        if (maxp <= 16) hipLaunchKernelGGL((step_kernel_coop_help<T, 16>), dim3((unsigned)blocks), dim3(2 * STEP_BLOCK), 0, s, LEAD_ARGS(p), p);
        else hipLaunchKernelGGL((step_kernel_coop_help<T, 32>), dim3((unsigned)blocks), dim3(2 * STEP_BLOCK), 0, s, LEAD_ARGS(p), p);
    } else if (coop) {
        if (maxp <= 16) hipLaunchKernelGGL((step_kernel_coop<T, 16>), dim3((unsigned)blocks), dim3(STEP_BLOCK), 0, s, LEAD_ARGS(p), p);
        else hipLaunchKernelGGL((step_kernel_coop<T, 32>), dim3((unsigned)blocks), dim3(STEP_BLOCK), 0, s, LEAD_ARGS(p), p);
    } else if (form == FORM_WIDE || form == FORM_WIDE_HELP) {
        const hipError_t we = launch_step_wide<T>(p, maxp, form == FORM_WIDE_HELP, s);
        if (we != hipSuccess) return we;
    } else {
        if (maxp <= 16) hipLaunchKernelGGL((step_kernel_one<T, 16>), dim3((unsigned)blocks), dim3(STEP_BLOCK), 0, s, LEAD_ARGS(p), p);
        else hipLaunchKernelGGL((step_kernel_one<T, 32>), dim3((unsigned)blocks), dim3(STEP_BLOCK), 0, s, LEAD_ARGS(p), p);
    }
    if (boxes) {
        const int64_t bb = (p.n_local + STEP_BLOCK - 1) / STEP_BLOCK;
        const unsigned nbb = (unsigned)(bb < 1 ? 1 : bb > 256 ? 256 : bb);
        if (maxp <= 16) hipLaunchKernelGGL((box_kernel<T, 16>), dim3(nbb), dim3(STEP_BLOCK), 0, s, p);
        else hipLaunchKernelGGL((box_kernel<T, 32>), dim3(nbb), dim3(STEP_BLOCK), 0, s, p);
    }
    return hipGetLastError();
}

// ---- the state across the boundary (rb_set_state / rb_get_state) ----------
// One lane per body: AoS rows of the caller (qpos[7k], qvel[6k], D1-fixed
// multi_sphere_bounce.py layout) <-> SoA state rows and snapshot.  The host
// moves the rows with one DMA each way (pinned staging, rb_capi.hip).
template <typename T>
__global__ __launch_bounds__(256) void state_in_kernel(StateIO<T> p) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.N) return;
    const double *q = p.qpos + 7 * b;
    p.snap[b] = Snap<T>{(T)q[0], (T)q[1], (T)q[2], p.bound[b]};
    if (p.quat) {
        T *o = p.quat + 4 * b;
        o[0] = (T)q[3]; o[1] = (T)q[4]; o[2] = (T)q[5]; o[3] = (T)q[6];
    }
    const int64_t l = b - p.lo;
    if (l < 0 || l >= p.n_local) return;
    const double *v = p.qvel + 6 * b;
#pragma unroll
    for (int d = 0; d < 4; ++d) p.st.row(d)[l] = (T)q[3 + d];
#pragma unroll
    for (int d = 0; d < 6; ++d) p.st.row(4 + d)[l] = (T)v[d];
#pragma unroll
    for (int d = 0; d < 3; ++d) p.st.row(10 + d)[l] = (T)q[d];
}

template <typename T>
__global__ __launch_bounds__(256) void state_out_kernel(StateIO<T> p, int want_q, int want_v) {
    const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= p.n_local) return;
    const int64_t b = p.lo + l;
    if (want_q) {
        double *q = p.qpos + 7 * b;
        if (p.balls) {
#pragma unroll
            for (int d = 0; d < 3; ++d) q[d] = (double)p.st.row(10 + d)[l];
        } else {
            const Snap<T> s = p.snap[b];
            q[0] = (double)s.x; q[1] = (double)s.y; q[2] = (double)s.z;
        }
#pragma unroll
        for (int d = 0; d < 4; ++d) q[3 + d] = (double)p.st.row(d)[l];
    }
    if (want_v) {
        double *v = p.qvel + 6 * b;
#pragma unroll
        for (int d = 0; d < 6; ++d) v[d] = (double)p.st.row(4 + d)[l];
    }
}

// The same rows written straight into mapped pinned host memory (p.qpos /
// p.qvel host-mapped): one lane per output double, so every wave's store is
// one contiguous 512 B run across PCIe (a lane per body would scatter 56 B
// strides); the SoA rows are gathered from HBM instead.
template <typename T>
__global__ __launch_bounds__(256) void state_out_flat_kernel(StateIO<T> p, int want_q, int want_v) {
    const int64_t nq = want_q ? 7 * (int64_t)p.n_local : 0, nv = want_v ? 6 * (int64_t)p.n_local : 0;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nq + nv; e += (int64_t)gridDim.x * blockDim.x) {
        if (e < nq) {
            const int64_t l = e / 7;
            const int d = (int)(e - 7 * l);
            T x;
            if (d >= 3) x = p.st.row(d - 3)[l];
            else if (p.balls) x = p.st.row(10 + d)[l];
            else x = reinterpret_cast<const T *>(p.snap + p.lo + l)[d];
            p.qpos[7 * p.lo + e] = (double)x;
        } else {
            const int64_t f = e - nq, l = f / 6;
            const int d = (int)(f - 6 * l);
            p.qvel[6 * p.lo + f] = (double)p.st.row(4 + d)[l];
        }
    }
}

template <typename T> hipError_t launch_state_in(const StateIO<T> &p, hipStream_t s) {
    if (p.N <= 0) return hipSuccess;
    hipLaunchKernelGGL((state_in_kernel<T>), dim3((unsigned)((p.N + 255) / 256)), dim3(256), 0, s, p);
    return hipGetLastError();
}
template <typename T> hipError_t launch_state_out(const StateIO<T> &p, bool want_q, bool want_v, hipStream_t s) {
    if (p.n_local <= 0) return hipSuccess;
    hipLaunchKernelGGL((state_out_kernel<T>), dim3((unsigned)((p.n_local + 255) / 256)), dim3(256), 0, s, p,
                       want_q ? 1 : 0, want_v ? 1 : 0);
    return hipGetLastError();
}
template <typename T> hipError_t launch_state_out_flat(const StateIO<T> &p, bool want_q, bool want_v, hipStream_t s) {
    if (p.n_local <= 0) return hipSuccess;
    const int64_t n = 13 * (int64_t)p.n_local;
    const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL((state_out_flat_kernel<T>), dim3(blocks), dim3(256), 0, s, p, want_q ? 1 : 0, want_v ? 1 : 0);
    return hipGetLastError();
}

template <typename T> hipError_t launch_insert(const InsertParams<T> &p, hipStream_t s) {
    if (p.count <= 0) return hipSuccess;
    const int64_t blocks = (p.count + 255) / 256;
    hipLaunchKernelGGL((insert_kernel<T>), dim3((unsigned)blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

template <typename T> hipError_t launch_kat_impulse(int64_t n, const double *in, double *out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL((kat_impulse_kernel<T>), dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, n, in, out);
    return hipGetLastError();
}

template <typename T> hipError_t launch_kat_inertia(int64_t n, const double *in, double *out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL((kat_inertia_kernel<T>), dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, n, in, out);
    return hipGetLastError();
}

template <typename T> hipError_t launch_kat_apply(int64_t n, const double *in, double *out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL((kat_apply_kernel<T>), dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, n, in, out);
    return hipGetLastError();
}

template <typename T> hipError_t launch_kat_narrow(int64_t n, const double *in, double *out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL((kat_narrow_kernel<T>), dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, n, in, out);
    return hipGetLastError();
}

template <typename T> hipError_t launch_step_wide(const StepParams<T> &p, int maxp, bool help, hipStream_t s) {
    int64_t blocks = (p.n_local + STEP_BLOCK - 1) / STEP_BLOCK;
    if (blocks < 1) blocks = 1;
    const bool halo = p.halo.mail != nullptr;
#define RB_WIDE_LAUNCH(K, M, H, TH)                                                                               \
    hipLaunchKernelGGL((K<T, M, H>), dim3((unsigned)blocks), dim3(TH), 0, s, LEAD_ARGS(p), p)
    if (help) {
        if (maxp <= 16) {
            if (halo) RB_WIDE_LAUNCH(step_kernel_wide_help, 16, true, 2 * STEP_BLOCK);
            else RB_WIDE_LAUNCH(step_kernel_wide_help, 16, false, 2 * STEP_BLOCK);
        } else {
            if (halo) RB_WIDE_LAUNCH(step_kernel_wide_help, 32, true, 2 * STEP_BLOCK);
            else RB_WIDE_LAUNCH(step_kernel_wide_help, 32, false, 2 * STEP_BLOCK);
        }
        return hipGetLastError();
    }
    if (maxp <= 16) {
        if (halo) RB_WIDE_LAUNCH(step_kernel_wide, 16, true, STEP_BLOCK);
        else RB_WIDE_LAUNCH(step_kernel_wide, 16, false, STEP_BLOCK);
    } else {
        if (halo) RB_WIDE_LAUNCH(step_kernel_wide, 32, true, STEP_BLOCK);
        else RB_WIDE_LAUNCH(step_kernel_wide, 32, false, STEP_BLOCK);
    }
#undef RB_WIDE_LAUNCH
    return hipGetLastError();
}

// explicit instantiations: RB_INST bit 1 = fp64, bit 2 = fp32 (the Makefile
// builds the two halves as separate objects, in parallel); RB_WIDE_UNIT: the
// wide form's kernel only (compiled with its own scheduling flags), else
// everything else
#ifndef RB_INST
#define RB_INST 3
#endif
#ifndef RB_WIDE_UNIT
#define RB_WIDE_UNIT 2                  // both (a one-command build of all sources)
#endif
#if RB_WIDE_UNIT >= 1 && (RB_INST & 1)
template hipError_t launch_step_wide<double>(const StepParams<double> &, int, bool, hipStream_t);
#endif
#if RB_WIDE_UNIT >= 1 && (RB_INST & 2)
template hipError_t launch_step_wide<float>(const StepParams<float> &, int, bool, hipStream_t);
#endif
#if RB_WIDE_UNIT != 1 && (RB_INST & 1)
template hipError_t launch_step<double>(const StepParams<double> &, int, int, bool, hipStream_t);
template hipError_t launch_kat_narrow<double>(int64_t, const double *, double *, hipStream_t);
template hipError_t launch_insert<double>(const InsertParams<double> &, hipStream_t);
template hipError_t launch_state_in<double>(const StateIO<double> &, hipStream_t);
template hipError_t launch_state_out<double>(const StateIO<double> &, bool, bool, hipStream_t);
template hipError_t launch_state_out_flat<double>(const StateIO<double> &, bool, bool, hipStream_t);
template hipError_t launch_kat_impulse<double>(int64_t, const double *, double *, hipStream_t);
template hipError_t launch_kat_inertia<double>(int64_t, const double *, double *, hipStream_t);
template hipError_t launch_kat_apply<double>(int64_t, const double *, double *, hipStream_t);
#endif
#if RB_WIDE_UNIT != 1 && (RB_INST & 2)
template hipError_t launch_step<float>(const StepParams<float> &, int, int, bool, hipStream_t);
template hipError_t launch_kat_narrow<float>(int64_t, const double *, double *, hipStream_t);
template hipError_t launch_insert<float>(const InsertParams<float> &, hipStream_t);
template hipError_t launch_state_in<float>(const StateIO<float> &, hipStream_t);
template hipError_t launch_state_out<float>(const StateIO<float> &, bool, bool, hipStream_t);
template hipError_t launch_state_out_flat<float>(const StateIO<float> &, bool, bool, hipStream_t);
template hipError_t launch_kat_impulse<float>(int64_t, const double *, double *, hipStream_t);
template hipError_t launch_kat_inertia<float>(int64_t, const double *, double *, hipStream_t);
template hipError_t launch_kat_apply<float>(int64_t, const double *, double *, hipStream_t);
#endif

}  // namespace rb
