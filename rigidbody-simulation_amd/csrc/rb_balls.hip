// rb_balls.hip — the reference's second contact law on gfx950: the
// symmetric two-ball impulse of src/simulation/ball_collision.py.
//
//   compute_inverse_inertia  :39-41   I_inv = eye(3) / ((2/5) m r^2)
//   compute_collision_impulse :53-68  full effective mass 1/m + n.((I^-1 (r x n)) x r),
//                                     friction clipped to mu |jn|
//   step_with_custom_collisions :73-125
//     gravity v += g dt; ground contact against z = 0 when z < r (impulse,
//     then z = r); ball-ball contact when |p2 - p1| < 2r + tol (the impulse
//     from ball 1's side, applied + to ball 1 and - to ball 2, positions
//     pushed apart by half the overlap); x += v dt; the quaternion is never
//     touched.
//
// The reference has two balls.  For N balls every pair (a < b) within
// r_a + r_b + tol is evaluated from the post-ground state of both (Jacobi
// over pairs) and each ball accumulates its pairs' deltas in ascending
// partner id — exactly the reference step for two balls (the oracle,
// oracle/rb_oracle_pairs.h, restates the same definition).
//
// One launch per step, one lane per ball.  A ball's ground phase depends on
// its own state only, so the step that finishes a ball also runs the ground
// phase of the NEXT step on it: the snapshots (and Vel records) hold post-
// ground positions / velocities, which is what the pair phase and the
// broadphase read; the true end-of-step state is kept in BodyState
// (px, py, pz, v, w).  The world re-runs the ground phase (ball_prime_kernel)
// whenever dt, e or mu change or the state is set.
#include "rb_device.hpp"
#include "rb_grid.hpp"
#include "rb_internal.hpp"

namespace rb {

// ball_collision.py:53-68
template <typename T>
__device__ __forceinline__ V3<T> pair_impulse(T mass, const M3<T> &Iinv, V3<T> v, V3<T> w, V3<T> r, V3<T> n, T e,
                                              T mu) {
    const V3<T> c = np_cross(w, r);
    const V3<T> vc = {v.x + c.x, v.y + c.y, v.z + c.z};                     // :54
    const T vn = np_dot(vc, n);                                             // :55
    const V3<T> vt = {vc.x - vn * n.x, vc.y - vn * n.y, vc.z - vn * n.z};   // :56
    const T tn = sqroot(np_dot(vt, vt));                                    // :57
    const V3<T> axr = np_cross(np_matvec(Iinv, np_cross(r, n)), r);
    const T dn = (T(1) / mass) + np_dot(n, axr);                            // :59
    const T jn = (-(T(1) + e) * vn) / dn;                                   // :60
    V3<T> td = {T(0), T(0), T(0)};
    if (tn > T(1e-8)) td = {vt.x / tn, vt.y / tn, vt.z / tn};               // :62
    const V3<T> bxr = np_cross(np_matvec(Iinv, np_cross(r, td)), r);
    const T dtn = (T(1) / mass) + np_dot(td, bxr);                          // :63-64
    const T jtu = -tn / dtn;                                                // :65
    const T lim = mu * absval(jn);
    T jt = jtu > -lim ? jtu : -lim;                                         // :66 np.clip
    jt = jt < lim ? jt : lim;
    return {jn * n.x + jt * td.x, jn * n.y + jt * td.y, jn * n.z + jt * td.z};   // :68
}

// ball_collision.py:39-41
template <typename T> __device__ __forceinline__ M3<T> ball_iinv(T m, T r) {
    const T I = (T(0.4) * m) * (r * r);
    M3<T> A;
#pragma unroll
    for (int k = 0; k < 9; ++k) A.a[k] = (k % 4 == 0) ? T(1) / I : T(0) / I;
    return A;
}

// gravity and the ground contact of one ball (ball_collision.py:77-97)
template <typename T>
__device__ __forceinline__ void ball_ground(const StepParams<T> &p, V3<T> &x, V3<T> &v, V3<T> &w, T m, T rad,
                                            const M3<T> &Iinv) {
    v = {v.x + p.g[0] * p.dt, v.y + p.g[1] * p.dt, v.z + p.g[2] * p.dt};   // :78
    if (!p.ground || !(x.z < rad)) return;                                  // :90
    const V3<T> n = {T(0), T(0), T(1)};                                     // :88
    const V3<T> cp = {x.x - rad * n.x, x.y - rad * n.y, x.z - rad * n.z};   // :91
    const V3<T> rr = {cp.x - x.x, cp.y - x.y, cp.z - x.z};                  // :92
    const V3<T> imp = pair_impulse(m, Iinv, v, w, rr, n, p.e, p.mu);        // :93-94
    const V3<T> dw = np_matvec(Iinv, np_cross(rr, imp));
    v = {v.x + imp.x / m, v.y + imp.y / m, v.z + imp.z / m};                // :95
    w = {w.x + dw.x, w.y + dw.y, w.z + dw.z};                               // :96
    x.z = rad;                                                              // :97
}

// |p_b - p_a| < r_a + r_b + tol for the pair (a < b), ball_collision.py:100-103
// (decided on the squared distance when clear of the threshold, see
// sphere_sphere_hit)
template <typename T> __device__ __forceinline__ bool ball_hit(V3<T> pa, T ra, V3<T> pb, T rb, T tol) {
    const V3<T> d = {pb.x - pa.x, pb.y - pa.y, pb.z - pa.z};
    const T d2 = np_dot(d, d);
    const T L = (ra + rb) + tol;
    const T L2 = L * L;
    if (RB_SQ_PREFILTER) {
        if (d2 > L2 * (T(1) + sq_margin<T>())) return false;
        if (d2 < L2 * (T(1) - sq_margin<T>())) return true;
    }
    return sqroot(d2) < L;
}

template <typename T, int MAXP>
__device__ __forceinline__ void ball_body(const StepParams<T> &p, int32_t l, int tid, int32_t *s_id, uint32_t gen) {
    const int32_t i = p.lo + l;
    const Snap<T> own = p.snap_cur[i];            // post-ground position, radius
    const Vel<T> ov = p.vel_cur[i];
    const V3<T> xo = {own.x, own.y, own.z};
    const V3<T> vo = {ov.vx, ov.vy, ov.vz}, wo = {ov.wx, ov.wy, ov.wz};
    const T mi = p.cs.mass()[i], ri = own.r;
    const M3<T> Ii = ball_iinv(mi, ri);

    // pairs: every partner within reach on the post-ground positions
    const int32_t np_ = search_buckets<T, MAXP>(p, i, xo, s_id, tid, gen, [&](uint32_t tj, const Snap<T> &s) {
        const int32_t j = (int32_t)(tj & ~BOX_FLAG);
        if (j == i) return false;
        const V3<T> xj = {s.x, s.y, s.z};
        return i < j ? ball_hit(xo, ri, xj, s.r, p.tol) : ball_hit(xj, s.r, xo, ri, p.tol);
    });

    // each pair from the post-ground state of both balls, deltas accumulated
    // in ascending partner id (ball_collision.py:100-118)
    V3<T> x = xo, v = vo, w = wo;
    int32_t nrec = 0;
    for (int s = 0; s < np_; ++s) {
        const int32_t j = s_id[s * STEP_BLOCK + tid];
        const Snap<T> sj = p.snap_cur[j];
        const Vel<T> vj = p.vel_cur[j];
        const V3<T> xj = {sj.x, sj.y, sj.z};
        const T mj = p.cs.mass()[j];
        const bool self_a = i < j;
        const V3<T> pa = self_a ? xo : xj, pb = self_a ? xj : xo;
        const V3<T> va = self_a ? vo : V3<T>{vj.vx, vj.vy, vj.vz};
        const V3<T> wa = self_a ? wo : V3<T>{vj.wx, vj.wy, vj.wz};
        const T ma = self_a ? mi : mj, ra = self_a ? ri : sj.r, rb = self_a ? sj.r : ri;
        const M3<T> Ia = self_a ? Ii : ball_iinv(mj, sj.r);
        const V3<T> diff = {pb.x - pa.x, pb.y - pa.y, pb.z - pa.z};         // :100
        const T dist = sqroot(np_dot(diff, diff));                          // :101
        const T dd = dist + T(1e-8);
        const V3<T> n = {diff.x / dd, diff.y / dd, diff.z / dd};            // :104
        const V3<T> cp = {(pa.x + pb.x) / T(2), (pa.y + pb.y) / T(2), (pa.z + pb.z) / T(2)};   // :105
        const V3<T> r1 = {cp.x - pa.x, cp.y - pa.y, cp.z - pa.z};           // :106
        const V3<T> imp = pair_impulse(ma, Ia, va, wa, r1, n, p.e, p.mu);   // :109-110
        const T corr = (((ra + rb) + p.tol) - dist) / T(2);                 // :116
        if (p.rec_count) {
            if (nrec < p.maxrec) {
                const int64_t o = (int64_t)l * p.maxrec + nrec;
                p.rec_partner[o] = j;
                p.rec_kind[o] = 16;
                p.rec_dist[o] = dist;
            }
            ++nrec;
        }
        if (self_a) {
            const V3<T> dw = np_matvec(Ii, np_cross(r1, imp));
            v = {v.x + imp.x / mi, v.y + imp.y / mi, v.z + imp.z / mi};     // :111
            w = {w.x + dw.x, w.y + dw.y, w.z + dw.z};                       // :112
            x = {x.x - corr * n.x, x.y - corr * n.y, x.z - corr * n.z};     // :117
        } else {
            const V3<T> r2 = {cp.x - pb.x, cp.y - pb.y, cp.z - pb.z};       // :107
            const V3<T> dw = np_matvec(Ii, np_cross(r2, imp));
            v = {v.x - imp.x / mi, v.y - imp.y / mi, v.z - imp.z / mi};     // :113
            w = {w.x - dw.x, w.y - dw.y, w.z - dw.z};                       // :114
            x = {x.x + corr * n.x, x.y + corr * n.y, x.z + corr * n.z};     // :118
        }
    }
    if (p.rec_count) p.rec_count[l] = nrec;

    // integrate (:121-122): the true end-of-step state
    x = {x.x + v.x * p.dt, x.y + v.y * p.dt, x.z + v.z * p.dt};
    wt_store(p.st.px() + l, x.x); wt_store(p.st.py() + l, x.y); wt_store(p.st.pz() + l, x.z);
    wt_store(p.st.vx() + l, v.x); wt_store(p.st.vy() + l, v.y); wt_store(p.st.vz() + l, v.z);
    wt_store(p.st.wx() + l, w.x); wt_store(p.st.wy() + l, w.y); wt_store(p.st.wz() + l, w.z);

    // the next step's ground phase, then its snapshot and broadphase slot
    ball_ground(p, x, v, w, mi, ri, Ii);
    Snap<T> sn;
    sn.x = x.x; sn.y = x.y; sn.z = x.z; sn.r = ri;
    Claim cl{0u, 0, 0ull, 0u, 0};
    if (p.next.line) cl = claim_slot(p.grid, p.next, p.err, sn, gen + 1u);
    wt_store(p.snap_next + i, sn);
    Vel<T> vn;
    vn.vx = v.x; vn.vy = v.y; vn.vz = v.z; vn.wx = w.x; vn.wy = w.y; vn.wz = w.z; vn.pad0 = T(0); vn.pad1 = T(0);
    p.vel_next[i] = vn;
    publish_slot(p.next, p.err, cl, sn, (uint32_t)i);
}

template <typename T, int MAXP>
__global__ __launch_bounds__(STEP_BLOCK) void ball_step_kernel(StepParams<T> p) {
    __shared__ int32_t s_id[MAXP * STEP_BLOCK];
    const int tid = threadIdx.x;
    const int64_t gt = (int64_t)blockIdx.x * STEP_BLOCK + tid;
    // generations: see step_body
    const uint32_t gen = *p.cur.gen;
    if (p.next.line && blockIdx.x == 0 && tid == 0) *p.next.gen = gen + 1u;
    if (gt < p.n_local) ball_body<T, MAXP>(p, (int32_t)gt, tid, s_id, gen);
}

// Ground phase of the coming step from the true state: post-ground snapshot
// and Vel record of every owned ball (into p.snap_next / p.vel_next).
template <typename T>
__global__ __launch_bounds__(256) void ball_prime_kernel(StepParams<T> p) {
    const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= p.n_local) return;
    const int32_t i = p.lo + (int32_t)l;
    V3<T> x = {p.st.px()[l], p.st.py()[l], p.st.pz()[l]};
    V3<T> v = {p.st.vx()[l], p.st.vy()[l], p.st.vz()[l]};
    V3<T> w = {p.st.wx()[l], p.st.wy()[l], p.st.wz()[l]};
    const T m = p.cs.mass()[i], r = p.cs.sx()[i];
    ball_ground(p, x, v, w, m, r, ball_iinv(m, r));
    Snap<T> sn;
    sn.x = x.x; sn.y = x.y; sn.z = x.z; sn.r = r;
    p.snap_next[i] = sn;
    Vel<T> vn;
    vn.vx = v.x; vn.vy = v.y; vn.vz = v.z; vn.wx = w.x; vn.wy = w.y; vn.wz = w.z; vn.pad0 = T(0); vn.pad1 = T(0);
    p.vel_next[i] = vn;
}

// KAT: in[27] = m, e, mu, v3, w3, r3, n3, I_inv9 -> out[3]
template <typename T>
__global__ void kat_pair_impulse_kernel(int64_t n, const double *in, double *out) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const double *a = in + 27 * c;
    M3<T> I;
#pragma unroll
    for (int k = 0; k < 9; ++k) I.a[k] = (T)a[15 + k];
    const V3<T> imp = pair_impulse((T)a[0], I, V3<T>{(T)a[3], (T)a[4], (T)a[5]}, V3<T>{(T)a[6], (T)a[7], (T)a[8]},
                                   V3<T>{(T)a[9], (T)a[10], (T)a[11]}, V3<T>{(T)a[12], (T)a[13], (T)a[14]},
                                   (T)a[1], (T)a[2]);
    out[3 * c] = (double)imp.x; out[3 * c + 1] = (double)imp.y; out[3 * c + 2] = (double)imp.z;
}

template <typename T> hipError_t launch_ball_step(const StepParams<T> &p, int maxp, hipStream_t s) {
    if (!p.vel_cur || !p.vel_next || !p.st.px()) return hipErrorInvalidValue;
    int64_t blocks = (p.n_local + STEP_BLOCK - 1) / STEP_BLOCK;
    if (blocks < 1) blocks = 1;
    if (maxp <= 16) hipLaunchKernelGGL((ball_step_kernel<T, 16>), dim3((unsigned)blocks), dim3(STEP_BLOCK), 0, s, p);
    else hipLaunchKernelGGL((ball_step_kernel<T, 32>), dim3((unsigned)blocks), dim3(STEP_BLOCK), 0, s, p);
    return hipGetLastError();
}

template <typename T> hipError_t launch_ball_prime(const StepParams<T> &p, hipStream_t s) {
    if (!p.vel_next || !p.st.px()) return hipErrorInvalidValue;
    if (p.n_local <= 0) return hipSuccess;
    hipLaunchKernelGGL((ball_prime_kernel<T>), dim3((unsigned)((p.n_local + 255) / 256)), dim3(256), 0, s, p);
    return hipGetLastError();
}

template <typename T> hipError_t launch_kat_pair_impulse(int64_t n, const double *in, double *out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL((kat_pair_impulse_kernel<T>), dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, n, in, out);
    return hipGetLastError();
}

template hipError_t launch_ball_step<double>(const StepParams<double> &, int, hipStream_t);
template hipError_t launch_ball_step<float>(const StepParams<float> &, int, hipStream_t);
template hipError_t launch_ball_prime<double>(const StepParams<double> &, hipStream_t);
template hipError_t launch_ball_prime<float>(const StepParams<float> &, hipStream_t);
template hipError_t launch_kat_pair_impulse<double>(int64_t, const double *, double *, hipStream_t);
template hipError_t launch_kat_pair_impulse<float>(int64_t, const double *, double *, hipStream_t);

}  // namespace rb
