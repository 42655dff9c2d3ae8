// rb_device.hpp — device-side arithmetic of the stepper (gfx950).
//
// Every function here keeps the operation order of the reference's
// NumPy/SciPy arithmetic (as executed on the golden machine: FMA-chain
// dot/norm/gemm, OpenBLAS getf2/getrs inverse) or of MuJoCo's C helpers
// (plain left-to-right), so that the fp64 path reproduces the reference
// bit for bit.  The translation unit is compiled with -ffp-contract=off:
// every fused multiply-add below is an explicit fmaf/fma, nothing else fuses.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rb {

__device__ __forceinline__ double fmadd(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float fmadd(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double sqroot(double a) { return __builtin_sqrt(a); }
__device__ __forceinline__ float sqroot(float a) { return __builtin_sqrtf(a); }
__device__ __forceinline__ double absval(double a) { return __builtin_fabs(a); }
__device__ __forceinline__ float absval(float a) { return __builtin_fabsf(a); }

template <typename T> struct V3 { T x, y, z; };
template <typename T> struct Q4 { T w, x, y, z; };
template <typename T> struct M3 { T a[9]; };   // row-major

// ---- NumPy / OpenBLAS semantics (collision.py, physics_utils.py) ---------
template <typename T> __device__ __forceinline__ T np_dot(V3<T> a, V3<T> b) {
    return fmadd(a.z, b.z, fmadd(a.y, b.y, a.x * b.x));
}
template <typename T> __device__ __forceinline__ V3<T> np_cross(V3<T> a, V3<T> b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// (3,3) @ (3,): fma(a2, x2, fma(a0, x0, a1*x1)) per row
template <typename T> __device__ __forceinline__ V3<T> np_matvec(const M3<T>& A, V3<T> v) {
    return {fmadd(A.a[2], v.z, fmadd(A.a[0], v.x, A.a[1] * v.y)),
            fmadd(A.a[5], v.z, fmadd(A.a[3], v.x, A.a[4] * v.y)),
            fmadd(A.a[8], v.z, fmadd(A.a[6], v.x, A.a[7] * v.y))};
}

// inverse of a 3x3 (np.linalg.inv -> getf2 + getrs), fully unrolled so the
// pivot state stays in registers.
template <typename T> __device__ __forceinline__ void swp(T& a, T& b) { T t = a; a = b; b = t; }

template <typename T> __device__ M3<T> np_inv3(const M3<T>& A) {
    T a00 = A.a[0], a01 = A.a[1], a02 = A.a[2];
    T a10 = A.a[3], a11 = A.a[4], a12 = A.a[5];
    T a20 = A.a[6], a21 = A.a[7], a22 = A.a[8];
    // column 0: pivot search, row swap of column 0, scale
    int p0 = 0;
    {
        T b = absval(a00);
        if (absval(a10) > b) { b = absval(a10); p0 = 1; }
        if (absval(a20) > b) { p0 = 2; }
    }
    if (p0 == 1) swp(a00, a10); else if (p0 == 2) swp(a00, a20);
    { const T r = T(1) / a00; a10 = a10 * r; a20 = a20 * r; }
    // column 1: apply pivot 0, gemv update of rows 1..2, pivot, swap cols 0..1, scale
    if (p0 == 1) swp(a01, a11); else if (p0 == 2) swp(a01, a21);
    a11 = a11 - a10 * a01;
    a21 = a21 - a20 * a01;
    int p1 = 1;
    if (absval(a21) > absval(a11)) p1 = 2;
    {
        const T piv = (p1 == 2) ? a21 : a11;
        const T r = T(1) / piv;
        if (p1 == 2) { swp(a10, a20); swp(a11, a21); }
        a21 = a21 * r;
    }
    // column 2: apply pivots 0 and 1, trsv (row 1), gemv (row 2)
    if (p0 == 1) swp(a02, a12); else if (p0 == 2) swp(a02, a22);
    if (p1 == 2) swp(a12, a22);
    a12 = a12 - a10 * a02;
    { const T t = fmadd(a21, a12, a20 * a02); a22 = a22 - t; }
    // getrs: B = P I (sequential row swaps), then unit-L forward, U backward.
    // The permutation only moves the unit entries: track which identity row
    // sits at rows 0..2.
    int r0 = 0, r1 = 1, r2 = 2;
    if (p0 == 1) swp(r0, r1); else if (p0 == 2) swp(r0, r2);
    if (p1 == 2) swp(r1, r2);
    M3<T> out;
#pragma unroll
    for (int col = 0; col < 3; ++col) {
        T b0 = (r0 == col) ? T(1) : T(0);
        T b1 = (r1 == col) ? T(1) : T(0);
        T b2 = (r2 == col) ? T(1) : T(0);
        b1 = fmadd(-b0, a10, b1);
        b2 = fmadd(-b0, a20, b2);
        b2 = fmadd(-b1, a21, b2);
        b2 = b2 * (T(1) / a22);
        b0 = b0 - a02 * b2;
        b1 = b1 - a12 * b2;
        b1 = b1 * (T(1) / a11);
        b0 = fmadd(-b1, a01, b0);
        b0 = b0 * (T(1) / a00);
        out.a[col] = b0; out.a[3 + col] = b1; out.a[6 + col] = b2;
    }
    return out;
}

// compute_inertia_tensor_world (collision.py:51-53): SciPy Rotation from
// (x,y,z,w) = q[[1,2,3,0]] (plain-sum normalisation, division), as_matrix,
// R @ diag(I) @ R.T with the OpenBLAS gemm order.
template <typename T> __device__ M3<T> inertia_world(V3<T> I, Q4<T> q) {
    T x = q.x, y = q.y, z = q.z, w = q.w;
    const T n = sqroot(((x * x + y * y) + z * z) + w * w);
    x = x / n; y = y / n; z = z / n; w = w / n;
    const T x2 = x * x, y2 = y * y, z2 = z * z, w2 = w * w;
    const T xy = x * y, zw = z * w, xz = x * z, yw = y * w, yz = y * z, xw = x * w;
    T R[9];
    R[0] = ((x2 - y2) - z2) + w2;   R[1] = T(2) * (xy - zw);          R[2] = T(2) * (xz + yw);
    R[3] = T(2) * (xy + zw);        R[4] = ((-x2 + y2) - z2) + w2;    R[5] = T(2) * (yz - xw);
    R[6] = T(2) * (xz - yw);        R[7] = T(2) * (yz + xw);          R[8] = ((-x2 - y2) + z2) + w2;
    // M = R @ diag(I): the gemm FMA chain over k with the zero entries kept
    const T D[9] = {I.x, T(0), T(0), T(0), I.y, T(0), T(0), T(0), I.z};
    T M[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            M[3 * i + j] = fmadd(R[3 * i + 2], D[6 + j], fmadd(R[3 * i + 1], D[3 + j], R[3 * i] * D[j]));
    M3<T> Iw;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            Iw.a[3 * i + j] = fmadd(M[3 * i + 2], R[3 * j + 2], fmadd(M[3 * i + 1], R[3 * j + 1], M[3 * i] * R[3 * j]));
    return Iw;
}

// compute_collision_impulse_friction (collision.py:7-48) then
// apply_impulse_friction (physics_utils.py:25-49) on one contact.
// Returns false (and leaves v, w untouched) when the contact separates
// (u_rel_n >= 0: the reference's zero impulse changes nothing but the sign
// of zeros).  jn/jt are exported for the KAT entry.
// k = 1/m + 1/18 (collision.py:35): a body constant, evaluated
// once per body-step instead of once per contact (the same value)
template <typename T> __device__ __forceinline__ T impulse_k(T m) { return (T(1) / m) + (T(1) / T(18)); }

template <typename T>
__device__ __forceinline__ bool impulse(T k, V3<T> v, V3<T> w, V3<T> r, V3<T> n, T e, T mu,
                                        T& jn_out, V3<T>& jt_out) {
    const V3<T> c = np_cross(w, r);
    const V3<T> u = {v.x + c.x, v.y + c.y, v.z + c.z};
    const T un = np_dot(u, n);
    const V3<T> ut = {u.x - un * n.x, u.y - un * n.y, u.z - un * n.z};
    jt_out = {T(0), T(0), T(0)};
    if (un >= T(0)) { jn_out = T(0); return false; }
    const T jn = (-(T(1) + e) * un) / k;
    const T nut = sqroot(np_dot(ut, ut));
    if (nut > T(1e-6)) {
        const T mf = mu * absval(jn);
        const T s = -((nut < mf) ? nut : mf);
        jt_out = {s * (ut.x / nut), s * (ut.y / nut), s * (ut.z / nut)};
    }
    jn_out = jn;
    return true;
}

template <typename T>
__device__ __forceinline__ void apply(V3<T>& v, V3<T>& w, T m, const M3<T>& invI, V3<T> r, V3<T> n,
                                      T jn, V3<T> jt) {
    const V3<T> P = {jn * n.x + jt.x, jn * n.y + jt.y, jn * n.z + jt.z};
    const V3<T> dw = np_matvec(invI, np_cross(r, P));
    v = {v.x + P.x / m, v.y + P.y / m, v.z + P.z / m};
    w = {w.x + dw.x, w.y + dw.y, w.z + dw.z};
}

// ---- MuJoCo semantics (contact generation, quaternion integration) --------
template <typename T> __device__ __forceinline__ T mj_dot(V3<T> a, V3<T> b) {
    return a.x * b.x + a.y * b.y + a.z * b.z;
}
template <typename T> __device__ __forceinline__ Q4<T> mj_mulquat(Q4<T> a, Q4<T> b) {
    return {a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z,
            a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
            a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
            a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w};
}
// free-joint kinematics: mju_normalize4 then mju_quat2Mat
template <typename T> __device__ M3<T> mj_body_mat(Q4<T> q) {
    const T nrm = sqroot(q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z);
    if (nrm < T(1e-15)) { q = {T(1), T(0), T(0), T(0)}; }
    else if (absval(nrm - T(1)) > T(1e-15)) {
        const T inv = T(1) / nrm;
        q = {q.w * inv, q.x * inv, q.y * inv, q.z * inv};
    }
    // mju_quat2Mat's identity shortcut, as selects (no early return)
    const bool ident = (q.w == T(1) && q.x == T(0) && q.y == T(0) && q.z == T(0));
    const T q00 = q.w * q.w, q01 = q.w * q.x, q02 = q.w * q.y, q03 = q.w * q.z;
    const T q11 = q.x * q.x, q12 = q.x * q.y, q13 = q.x * q.z;
    const T q22 = q.y * q.y, q23 = q.y * q.z, q33 = q.z * q.z;
    M3<T> M;
    M.a[0] = q00 + q11 - q22 - q33;
    M.a[4] = q00 - q11 + q22 - q33;
    M.a[8] = q00 - q11 - q22 + q33;
    M.a[1] = T(2) * (q12 - q03);
    M.a[2] = T(2) * (q13 + q02);
    M.a[3] = T(2) * (q12 + q03);
    M.a[5] = T(2) * (q23 - q01);
    M.a[6] = T(2) * (q13 - q02);
    M.a[7] = T(2) * (q23 + q01);
    if (ident) {
#pragma unroll
        for (int k = 0; k < 9; ++k) M.a[k] = (k % 4 == 0) ? T(1) : T(0);
    }
    return M;
}

template <typename T> struct Contact {
    T dist;
    V3<T> pos;
    V3<T> frame;    // geom1 -> geom2
};

// mjc_PlaneSphere
template <typename T>
__device__ __forceinline__ bool plane_sphere(V3<T> pn, V3<T> pp, V3<T> c, T rad, Contact<T>& con) {
    const V3<T> tmp = {c.x - pp.x, c.y - pp.y, c.z - pp.z};
    const T cdist = mj_dot(tmp, pn);
    if (cdist > T(0) + rad) return false;
    con.dist = cdist - rad;
    const T s = -con.dist / T(2) - rad;
    con.pos = {c.x + pn.x * s, c.y + pn.y * s, c.z + pn.z * s};
    con.frame = pn;
    return true;
}

// one corner of mjc_PlaneBox; `dist` = (c - p0).n of the box centre
template <typename T>
__device__ __forceinline__ bool plane_box_corner(V3<T> pn, V3<T> c, T dist, const M3<T>& M, V3<T> h,
                                                 int i, Contact<T>& con) {
    const V3<T> vec = {(i & 1) ? h.x : -h.x, (i & 2) ? h.y : -h.y, (i & 4) ? h.z : -h.z};
    V3<T> corner = {M.a[0] * vec.x + M.a[1] * vec.y + M.a[2] * vec.z,
                    M.a[3] * vec.x + M.a[4] * vec.y + M.a[5] * vec.z,
                    M.a[6] * vec.x + M.a[7] * vec.y + M.a[8] * vec.z};
    const T ldist = mj_dot(pn, corner);
    if (dist + ldist > T(0) || ldist > T(0)) return false;
    con.dist = dist + ldist;
    const T s = -con.dist / T(2);
    corner = {corner.x + c.x, corner.y + c.y, corner.z + c.z};
    con.pos = {corner.x + pn.x * s, corner.y + pn.y * s, corner.z + pn.z * s};
    con.frame = pn;
    return true;
}

// Relative margin under which a squared-distance comparison decides a
// distance test without the square root: far above the rounding of d^2 and
// R^2 (a few ulp), so the decision equals the exact sqrt(d^2) vs R one.
#ifndef RB_SQ_PREFILTER
#define RB_SQ_PREFILTER 1
#endif
template <typename T> __device__ __forceinline__ T sq_margin() { return sizeof(T) == 8 ? T(1e-9) : T(1e-4); }

// mjc_SphereSphere, geom1 = lower body id; test-only variant first.  Most
// candidates are clearly apart (or clearly overlapping): decided on d^2;
// the rest (and NaN) by the reference's sqrt comparison.
template <typename T>
__device__ __forceinline__ bool sphere_sphere_hit(V3<T> c1, T r1, V3<T> c2, T r2) {
    const V3<T> dif = {c1.x - c2.x, c1.y - c2.y, c1.z - c2.z};
    const T d2 = mj_dot(dif, dif);
    const T R = (T(0) + r1) + r2;
    const T R2 = R * R;
    if (RB_SQ_PREFILTER) {
        if (d2 > R2 * (T(1) + sq_margin<T>())) return false;
        if (d2 < R2 * (T(1) - sq_margin<T>())) return true;
    }
    return !(sqroot(d2) > R);
}
template <typename T>
__device__ __forceinline__ bool sphere_sphere(V3<T> c1, T r1, V3<T> c2, T r2, Contact<T>& con) {
    const V3<T> dif = {c1.x - c2.x, c1.y - c2.y, c1.z - c2.z};
    const T cdist = sqroot(mj_dot(dif, dif));
    if (cdist > (T(0) + r1) + r2) return false;
    con.dist = (cdist - r1) - r2;
    V3<T> f = {c2.x - c1.x, c2.y - c1.y, c2.z - c1.z};
    // |f| is cdist bit for bit: f = -dif exactly (round-to-nearest is
    // symmetric), so mj_dot(f, f) == mj_dot(dif, dif) — one square root less
    const T len = cdist;
    if (len < T(1e-15)) f = {T(1), T(0), T(0)};
    else { const T inv = T(1) / len; f = {f.x * inv, f.y * inv, f.z * inv}; }
    const T s = r1 + con.dist / T(2);
    con.pos = {f.x * s + c1.x, f.y * s + c1.y, f.z * s + c1.z};
    con.frame = f;
    return true;
}

}  // namespace rb
