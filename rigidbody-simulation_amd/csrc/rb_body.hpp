// rb_body.hpp — per-body pieces of the step shared by the hashed-cell step
// kernels (rb_kernels.hip) and the cell-ordered tile kernel (rb_tiles.hip):
// contact recording, the lazily evaluated world inverse inertia, one
// contact through the reference's skip rules and impulse (K2), gravity /
// applied forces (a4), and the integration of position and orientation
// (K3).  The operation order is the reference's (rb_device.hpp), so every
// kernel that calls these steps a body bit-identically.
#pragma once

#include "rb_device.hpp"
#include "rb_internal.hpp"

#ifndef RB_ABLATE
#define RB_ABLATE 0
#endif

namespace rb {

template <typename T>
__device__ __forceinline__ void record(const StepParams<T> &p, int32_t l, int32_t &nrec, int32_t partner,
                                       int32_t kind, T dist) {
    if (!p.rec_count) return;
    if (nrec < p.maxrec) {
        const int64_t o = (int64_t)l * p.maxrec + nrec;
        p.rec_partner[o] = partner;
        p.rec_kind[o] = kind;
        p.rec_dist[o] = dist;
    }
    ++nrec;
}

// Lazily evaluated inv(inertia_world): the reference computes it every step
// (collision.py:62) but it only reaches the state through a torque or an
// applied impulse; computing it on first use is value-identical and keeps
// it out of the broadphase's register live range.
template <typename T> struct LazyInvI {
    V3<T> I;
    Q4<T> q;
    bool have = false;
    M3<T> m;
    __device__ __forceinline__ const M3<T> &get() {
        if (!have) {
#if RB_ABLATE == 2
            for (int k = 0; k < 9; ++k) m.a[k] = (k % 4 == 0) ? T(1) / I.x : T(0);
#else
            m = np_inv3(inertia_world(I, q));
#endif
            have = true;
        }
        return m;
    }
};

// one contact of body i through the reference's skip rules then K2
template <typename T>
__device__ __forceinline__ void solve_contact(const StepParams<T> &p, const Contact<T> &con, V3<T> x, V3<T> n,
                                              T m, T k, LazyInvI<T> &invI, V3<T> &v, V3<T> &w) {
    if (!(con.dist < T(0))) return;                 // collision.py:74 (NaN fails too)
    if (absval(con.dist) < p.thr) return;           // collision.py:79-80
    const V3<T> r = {con.pos.x - x.x, con.pos.y - x.y, con.pos.z - x.z};   // :75
    T jn;
    V3<T> jt;
    if (impulse(k, v, w, r, n, p.e, p.mu, jn, jt)) apply(v, w, m, invI.get(), r, n, jn, jt);
}

// a4 (collision.py:66-70): gravity plus the optional applied force / torque
// (XFRC false: a caller whose worlds never carry one, so no branch on it)
template <typename T, bool XFRC = true>
__device__ __forceinline__ void apply_force(const StepParams<T> &p, int32_t l, T m, LazyInvI<T> &invI, V3<T> &v,
                                            V3<T> &w) {
    V3<T> F = {m * p.g[0], m * p.g[1], m * p.g[2]};
    if (XFRC && p.xfrc) F = {p.xfrc[l] + F.x, p.xfrc[p.S + l] + F.y, p.xfrc[2 * p.S + l] + F.z};
    v = {v.x + (F.x / m) * p.dt, v.y + (F.y / m) * p.dt, v.z + (F.z / m) * p.dt};
    if (XFRC && p.xfrc) {
        const V3<T> tdt = {p.xfrc[3 * p.S + l] * p.dt, p.xfrc[4 * p.S + l] * p.dt, p.xfrc[5 * p.S + l] * p.dt};
        const V3<T> dw = np_matvec(invI.get(), tdt);
        w = {w.x + dw.x, w.y + dw.y, w.z + dw.z};
    }
}

// K3 (collision.py:90-100): x += v dt; q += 0.5 (0, w) q dt, normalised —
// the same expressions as body_update's integration (rb_kernels.hip)
template <typename T>
__device__ __forceinline__ void integrate_pose(V3<T> &x, Q4<T> &qn, const Q4<T> &q, V3<T> v, V3<T> w, T dt) {
    x = {x.x + v.x * dt, x.y + v.y * dt, x.z + v.z * dt};
    const Q4<T> res = mj_mulquat(Q4<T>{T(0), w.x, w.y, w.z}, q);
    qn = {q.w + (T(0.5) * res.w) * dt, q.x + (T(0.5) * res.x) * dt, q.y + (T(0.5) * res.y) * dt,
          q.z + (T(0.5) * res.z) * dt};
    const T nq = sqroot(fmadd(qn.z, qn.z, fmadd(qn.y, qn.y, fmadd(qn.x, qn.x, qn.w * qn.w))));
    qn = {qn.w / nq, qn.x / nq, qn.y / nq, qn.z / nq};
}

}  // namespace rb
