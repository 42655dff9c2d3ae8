// rb_boxes.hpp — box-involved narrowphase on gfx950.
//
// MuJoCo's mjc_SphereBox / mjc_BoxBox are third-party C that is neither
// installed nor vendored in the build container, so these are this
// project's definitions, following the published structure of those
// primitives (margin 0; oracle/rb_oracle_impl.h "box pairs" states them and
// is the parity checker — parity against MuJoCo itself is unpinned):
//   sphere_box  sphere = geom1 (MuJoCo dispatches by geom type): the sphere
//               centre clamped to the box in the box frame; inside: the
//               nearest face;
//   box_box     separating-axis test over 15 axes (edge axes win only by a
//               1.05 factor), then either the incident face clipped against
//               the reference face (Sutherland-Hodgman, at most 4 points:
//               the deepest, in polygon order) or one edge-edge point.
// Every expression keeps the oracle's operation order (the translation unit
// is built with -ffp-contract=off), so fp64 results are bit-identical.
// Register arrays are only indexed by compile-time constants (selects
// instead of dynamic indices); the clipped polygon lives in LDS (a lane's
// 48 reals at stride `ps`), so the box kernels need no scratch.
#pragma once

#include "rb_device.hpp"
#include "rb_internal.hpp"

namespace rb {

template <typename T> __device__ __forceinline__ T clampv(T x, T lo, T hi) { return x < lo ? lo : (x > hi ? hi : x); }
template <typename T> __device__ __forceinline__ T sel3(int k, T a, T b, T c) { return k == 0 ? a : k == 1 ? b : c; }
template <typename T> __device__ __forceinline__ V3<T> sel3v(int k, V3<T> a, V3<T> b, V3<T> c) {
    return {sel3(k, a.x, b.x, c.x), sel3(k, a.y, b.y, c.y), sel3(k, a.z, b.z, c.z)};
}
template <typename T> __device__ __forceinline__ V3<T> mat_col(const M3<T> &M, int k) {
    return {M.a[k], M.a[3 + k], M.a[6 + k]};
}
template <typename T> __device__ __forceinline__ T comp(V3<T> v, int k) { return k == 0 ? v.x : k == 1 ? v.y : v.z; }

// sphere (c1, r1) = geom1, box (c2, M2, h2) = geom2
template <typename T>
__device__ __forceinline__ bool sphere_box(V3<T> c1, T r1, V3<T> c2, const M3<T> &M2, V3<T> h2, Contact<T> &con) {
    const V3<T> tmp = {c1.x - c2.x, c1.y - c2.y, c1.z - c2.z};
    const V3<T> center = {M2.a[0] * tmp.x + M2.a[3] * tmp.y + M2.a[6] * tmp.z,
                          M2.a[1] * tmp.x + M2.a[4] * tmp.y + M2.a[7] * tmp.z,
                          M2.a[2] * tmp.x + M2.a[5] * tmp.y + M2.a[8] * tmp.z};
    const V3<T> clamped = {clampv(center.x, -h2.x, h2.x), clampv(center.y, -h2.y, h2.y), clampv(center.z, -h2.z, h2.z)};
    const V3<T> nearest = {clamped.x - center.x, clamped.y - center.y, clamped.z - center.z};
    const T dist = sqroot(mj_dot(nearest, nearest));
    if (dist - r1 > T(0)) return false;
    V3<T> pos, nrm;
    T cd;
    if (dist <= T(1e-15)) {
        T closest = T(2) * ((h2.x + h2.y) + h2.z);
        int kf = 0;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const int a = i / 2;
            const T ha = comp(h2, a), ca = comp(center, a);
            const T df = (i % 2 == 0) ? ha - ca : ha + ca;
            if (df < closest) { closest = df; kf = i; }
        }
        const int a = kf / 2;
        const T s = (kf % 2 == 0) ? T(1) : T(-1);
        const T ca = sel3(a, center.x, center.y, center.z);
        const T pa = ca + s * ((closest - r1) / T(2));
        nrm = {a == 0 ? -s : T(0), a == 1 ? -s : T(0), a == 2 ? -s : T(0)};
        pos = {a == 0 ? pa : center.x, a == 1 ? pa : center.y, a == 2 ? pa : center.z};
        cd = -closest - r1;
    } else {
        const T inv = T(1) / dist;
        nrm = {nearest.x * inv, nearest.y * inv, nearest.z * inv};
        pos = {(clamped.x + (center.x + nrm.x * r1)) * T(0.5), (clamped.y + (center.y + nrm.y * r1)) * T(0.5),
               (clamped.z + (center.z + nrm.z * r1)) * T(0.5)};
        cd = dist - r1;
    }
    con.pos = {(M2.a[0] * pos.x + M2.a[1] * pos.y + M2.a[2] * pos.z) + c2.x,
               (M2.a[3] * pos.x + M2.a[4] * pos.y + M2.a[5] * pos.z) + c2.y,
               (M2.a[6] * pos.x + M2.a[7] * pos.y + M2.a[8] * pos.z) + c2.z};
    con.frame = {M2.a[0] * nrm.x + M2.a[1] * nrm.y + M2.a[2] * nrm.z,
                 M2.a[3] * nrm.x + M2.a[4] * nrm.y + M2.a[5] * nrm.z,
                 M2.a[6] * nrm.x + M2.a[7] * nrm.y + M2.a[8] * nrm.z};
    con.dist = cd;
    return true;
}

// box A (pa, Ma, ha) = geom1, box B = geom2.  emit(con, kind) is called for
// each contact in order (at most 4); returns the count.  poly: this lane's
// LDS polygon buffers, element e at poly[e * ps] (2 x 8 vertices x 3).
template <typename T, typename Emit>
__device__ __forceinline__ int box_box(V3<T> pa, const M3<T> &Ma, V3<T> ha, V3<T> pb, const M3<T> &Mb, V3<T> hb,
                                       T *poly, int ps, Emit emit) {
    V3<T> ua[3], ub[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) { ua[i] = mat_col(Ma, i); ub[i] = mat_col(Mb, i); }
    const V3<T> d = {pb.x - pa.x, pb.y - pa.y, pb.z - pa.z};
    T R[3][3], AR[3][3], da[3], db[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) { R[i][j] = mj_dot(ua[i], ub[j]); AR[i][j] = absval(R[i][j]); }
#pragma unroll
    for (int i = 0; i < 3; ++i) { da[i] = mj_dot(d, ua[i]); db[i] = mj_dot(d, ub[i]); }
    const T hav[3] = {ha.x, ha.y, ha.z}, hbv[3] = {hb.x, hb.y, hb.z};
    T best = T(0), dL = T(0);
    V3<T> L = {T(0), T(0), T(0)};
    int bk = -1;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const T s = absval(da[i]) - (hav[i] + ((hbv[0] * AR[i][0] + hbv[1] * AR[i][1]) + hbv[2] * AR[i][2]));
        if (s > T(0)) return 0;
        if (bk < 0 || s > best) { best = s; bk = i; }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const T s = absval(db[j]) - (((hav[0] * AR[0][j] + hav[1] * AR[1][j]) + hav[2] * AR[2][j]) + hbv[j]);
        if (s > T(0)) return 0;
        if (s > best) { best = s; bk = 3 + j; }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            V3<T> c = np_cross(ua[i], ub[j]);
            const T len = sqroot(mj_dot(c, c));
            if (len < T(1e-6)) continue;                       // parallel edges
            const T inv = T(1) / len;
            c = {c.x * inv, c.y * inv, c.z * inv};
            const T pA = (hav[0] * absval(mj_dot(ua[0], c)) + hav[1] * absval(mj_dot(ua[1], c))) +
                         hav[2] * absval(mj_dot(ua[2], c));
            const T pB = (hbv[0] * absval(mj_dot(ub[0], c)) + hbv[1] * absval(mj_dot(ub[1], c))) +
                         hbv[2] * absval(mj_dot(ub[2], c));
            const T dc = mj_dot(d, c);
            const T s = absval(dc) - (pA + pB);
            if (s > T(0)) return 0;
            if (s * T(1.05) > best) { best = s; bk = 6 + 3 * i + j; L = c; dL = dc; }
        }
    if (bk < 3) { L = sel3v(bk, ua[0], ua[1], ua[2]); dL = sel3(bk, da[0], da[1], da[2]); }
    else if (bk < 6) { L = sel3v(bk - 3, ub[0], ub[1], ub[2]); dL = sel3(bk - 3, db[0], db[1], db[2]); }
    const V3<T> n = dL < T(0) ? V3<T>{-L.x, -L.y, -L.z} : L;

    Contact<T> con;
    con.frame = n;
    if (bk >= 6) {                                             // edge - edge
        const int i = (bk - 6) / 3, j = (bk - 6) % 3;
        V3<T> qa = pa, qb = pb;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (k != i) {
                const T sg = mj_dot(ua[k], n) > T(0) ? hav[k] : -hav[k];
                qa = {qa.x + ua[k].x * sg, qa.y + ua[k].y * sg, qa.z + ua[k].z * sg};
            }
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (k != j) {
                const T sg = mj_dot(ub[k], n) > T(0) ? -hbv[k] : hbv[k];
                qb = {qb.x + ub[k].x * sg, qb.y + ub[k].y * sg, qb.z + ub[k].z * sg};
            }
        }
        const V3<T> r = {qb.x - qa.x, qb.y - qa.y, qb.z - qa.z};
        const V3<T> uai = sel3v(i, ua[0], ua[1], ua[2]), ubj = sel3v(j, ub[0], ub[1], ub[2]);
        const T a = sel3(i, sel3(j, R[0][0], R[0][1], R[0][2]), sel3(j, R[1][0], R[1][1], R[1][2]),
                         sel3(j, R[2][0], R[2][1], R[2][2]));
        const T e = mj_dot(uai, r), f = mj_dot(ubj, r);
        const T den = T(1) - a * a;
        const T hai = sel3(i, hav[0], hav[1], hav[2]), hbj = sel3(j, hbv[0], hbv[1], hbv[2]);
        const T s = clampv((e - a * f) / den, -hai, hai);
        const T t = clampv((a * e - f) / den, -hbj, hbj);
        con.pos = {((qa.x + uai.x * s) + (qb.x + ubj.x * t)) * T(0.5), ((qa.y + uai.y * s) + (qb.y + ubj.y * t)) * T(0.5),
                   ((qa.z + uai.z * s) + (qb.z + ubj.z * t)) * T(0.5)};
        con.dist = best;
        emit(con, CK_BOX_EDGE);
        return 1;
    }

    // face: reference box (the axis's owner), incident box (the other)
    const bool refa = bk < 3;
    const int ra = refa ? bk : bk - 3;
    const V3<T> pr = refa ? pa : pb, pi = refa ? pb : pa, hr = refa ? ha : hb, hi = refa ? hb : ha;
    V3<T> ur[3], ui[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) { ur[k] = refa ? ua[k] : ub[k]; ui[k] = refa ? ub[k] : ua[k]; }
    const V3<T> nr = refa ? n : V3<T>{-n.x, -n.y, -n.z};      // reference face normal, toward the incident box
    T cdot[3];
    int kk = 0;
    T cb = T(-1);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        cdot[k] = mj_dot(ui[k], nr);
        if (absval(cdot[k]) > cb) { cb = absval(cdot[k]); kk = k; }
    }
    const T sg = sel3(kk, cdot[0], cdot[1], cdot[2]) > T(0) ? T(-1) : T(1);
    const int b1 = kk == 0 ? 1 : 0, b2 = kk == 2 ? 1 : 2;
    const int a1 = ra == 0 ? 1 : 0, a2 = ra == 2 ? 1 : 2;
    const V3<T> uik = sel3v(kk, ui[0], ui[1], ui[2]), uib1 = sel3v(b1, ui[0], ui[1], ui[2]),
                uib2 = sel3v(b2, ui[0], ui[1], ui[2]);
    const V3<T> ura1 = sel3v(a1, ur[0], ur[1], ur[2]), ura2 = sel3v(a2, ur[0], ur[1], ur[2]);
    const T hik = sel3(kk, hi.x, hi.y, hi.z), hib1 = sel3(b1, hi.x, hi.y, hi.z), hib2 = sel3(b2, hi.x, hi.y, hi.z);
    const T hra = sel3(ra, hr.x, hr.y, hr.z), hra1 = sel3(a1, hr.x, hr.y, hr.z), hra2 = sel3(a2, hr.x, hr.y, hr.z);
    const T ssk = sg * hik;
    const V3<T> cinc = {pi.x + uik.x * ssk, pi.y + uik.y * ssk, pi.z + uik.z * ssk};
    const V3<T> e1 = {uib1.x * hib1, uib1.y * hib1, uib1.z * hib1};
    const V3<T> e2 = {uib2.x * hib2, uib2.y * hib2, uib2.z * hib2};
    const V3<T> cref = {pr.x + nr.x * hra, pr.y + nr.y * hra, pr.z + nr.z * hra};
    // polygon buffers: buf b, vertex v, coordinate c at poly[((b * 8 + v) * 3 + c) * ps]
    auto P = [&](int b, int v, int c) -> T & { return poly[((b * 8 + v) * 3 + c) * ps]; };
#pragma unroll
    for (int v = 0; v < 4; ++v) {                              // (+,+) (-,+) (-,-) (+,-)
        V3<T> vert = (v == 0 || v == 3) ? V3<T>{cinc.x + e1.x, cinc.y + e1.y, cinc.z + e1.z}
                                        : V3<T>{cinc.x - e1.x, cinc.y - e1.y, cinc.z - e1.z};
        vert = (v < 2) ? V3<T>{vert.x + e2.x, vert.y + e2.y, vert.z + e2.z}
                       : V3<T>{vert.x - e2.x, vert.y - e2.y, vert.z - e2.z};
        const V3<T> rel = {vert.x - cref.x, vert.y - cref.y, vert.z - cref.z};
        P(0, v, 0) = mj_dot(rel, ura1);
        P(0, v, 1) = mj_dot(rel, ura2);
        P(0, v, 2) = mj_dot(rel, nr);
    }
    int np = 4;
#pragma unroll
    for (int pl = 0; pl < 4; ++pl) {
        const int c = pl < 2 ? 0 : 1;
        const bool neg = pl & 1;
        const T w = pl < 2 ? hra1 : hra2;
        const int src = pl & 1, dst = 1 - src;
        int nq = 0;
        for (int t = 0; t < np; ++t) {
            const int tp = (t + np - 1) % np;
            const T cc = P(src, t, c), pc = P(src, tp, c);
            const T fc = (neg ? -cc : cc) - w;
            const T fp = (neg ? -pc : pc) - w;
            const bool ins = fc <= T(0), pins = fp <= T(0);
            if (ins != pins && nq < 8) {                       // the edge crosses the plane
                const T tt = fp / (fp - fc);
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const T pk = P(src, tp, k);
                    P(dst, nq, k) = pk + (P(src, t, k) - pk) * tt;
                }
                ++nq;
            }
            if (ins && nq < 8) {
#pragma unroll
                for (int k = 0; k < 3; ++k) P(dst, nq, k) = P(src, t, k);
                ++nq;
            }
        }
        np = nq;
    }
    // after 4 passes the polygon is back in buffer 0
    uint32_t keep = 0;
    int nk = 0;
    for (int t = 0; t < np; ++t)
        if (P(0, t, 2) <= T(0)) { keep |= 1u << t; ++nk; }
    if (nk > 4) {                                              // the 4 deepest
        uint32_t pick = 0;
        for (int r = 0; r < 4; ++r) {
            int bt = -1;
            T bz = T(0);
            for (int t = 0; t < np; ++t) {
                if (!(((keep & ~pick) >> t) & 1u)) continue;
                const T z = P(0, t, 2);
                if (bt < 0 || z < bz) { bt = t; bz = z; }
            }
            pick |= 1u << bt;
        }
        keep = pick;
    }
    int m = 0;
    for (int t = 0; t < np; ++t) {
        if (!((keep >> t) & 1u)) continue;
        const T x = P(0, t, 0), y = P(0, t, 1), z = P(0, t, 2), s = -z / T(2);
        const V3<T> wp = {((cref.x + ura1.x * x) + ura2.x * y) + nr.x * z, ((cref.y + ura1.y * x) + ura2.y * y) + nr.y * z,
                          ((cref.z + ura1.z * x) + ura2.z * y) + nr.z * z};
        con.pos = {wp.x + nr.x * s, wp.y + nr.y * s, wp.z + nr.z * s};
        con.dist = z;
        emit(con, CK_BOX_BOX0 + m);
        ++m;
    }
    return m;
}

}  // namespace rb
