/*
 * rb_oracle_impl.h — body of the CPU oracle, included twice by rb_oracle.c
 * (REAL=double, SFX=f64 and REAL=float, SFX=f32).
 *
 * TEST INFRASTRUCTURE ONLY.  This is a CPU restatement of the reference's
 * hot path, used as the parity checker by tests/, __graft_entry__.smoke()
 * and the cpu_baseline leg of bench.py.  The product path (librbhip.so)
 * never links, loads or calls it.
 *
 * Arithmetic contract (what makes the oracle bit-exact with the reference):
 *  - the reference's NumPy/SciPy arithmetic is restated in the exact
 *    operation order NumPy executes on the golden-generation machine
 *    (OpenBLAS 0.3.29 Haswell kernels, probed): dot/norm are FMA chains,
 *    3x3 matvec is fma(a2,x2, fma(a0,x0, a1*x1)), 3x3 gemm is an FMA chain
 *    over k = 0,1,2, np.linalg.inv is OpenBLAS getf2+getrs, SciPy's
 *    Rotation normalises with a plain sum and a division;
 *  - MuJoCo's C helpers (contact primitives, mju_mulQuat, mju_quat2Mat,
 *    mju_normalize4) are restated with plain left-to-right arithmetic.
 *  Compiled with -ffp-contract=off so the compiler adds no FMA of its own.
 */

#define CAT_(a, b) a##_##b
#define CAT(a, b) CAT_(a, b)
#define FN(name) CAT(name, SFX)

/* ---------------- NumPy / OpenBLAS restatements ------------------------- */
/* np.dot(a, b) for float64[3] (OpenBLAS ddot: FMA chain) */
static inline REAL FN(np_dot3)(const REAL a[3], const REAL b[3]) {
    return FMA(a[2], b[2], FMA(a[1], b[1], a[0] * b[0]));
}
/* np.linalg.norm(a) for float64[3] = sqrt(dot(a, a)) */
static inline REAL FN(np_norm3)(const REAL a[3]) { return SQRT(FN(np_dot3)(a, a)); }
/* np.linalg.norm(q) for float64[4] */
static inline REAL FN(np_norm4)(const REAL q[4]) {
    return SQRT(FMA(q[3], q[3], FMA(q[2], q[2], FMA(q[1], q[1], q[0] * q[0]))));
}
/* (3,3) @ (3,) — OpenBLAS dgemv_t small-size kernel order */
static inline void FN(np_matvec3)(const REAL A[9], const REAL x[3], REAL y[3]) {
    for (int i = 0; i < 3; ++i)
        y[i] = FMA(A[3 * i + 2], x[2], FMA(A[3 * i + 0], x[0], A[3 * i + 1] * x[1]));
}
/* (3,3) @ (3,3) — OpenBLAS dgemm order; bt!=0 means B is used transposed */
static inline void FN(np_gemm3)(const REAL A[9], const REAL B[9], int bt, REAL C[9]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            const REAL b0 = bt ? B[3 * j + 0] : B[0 * 3 + j];
            const REAL b1 = bt ? B[3 * j + 1] : B[1 * 3 + j];
            const REAL b2 = bt ? B[3 * j + 2] : B[2 * 3 + j];
            C[3 * i + j] = FMA(A[3 * i + 2], b2, FMA(A[3 * i + 1], b1, A[3 * i + 0] * b0));
        }
}
/* np.cross(a, b) for float64[3]: elementwise multiply + subtract */
static inline void FN(np_cross)(const REAL a[3], const REAL b[3], REAL c[3]) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}
/* np.linalg.inv for a 3x3 (numpy -> dgesv(A, I) -> OpenBLAS getf2 + getrs).
 * A, Ai row-major. */
static void FN(np_inv3)(const REAL A[9], REAL Ai[9]) {
    REAL a[3][3];
    int piv[3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) a[i][j] = A[3 * i + j];
    for (int j = 0; j < 3; ++j) {
        for (int i = 0; i < j; ++i) {            /* apply earlier pivots to column j */
            const int p = piv[i];
            if (p != i) { REAL t = a[i][j]; a[i][j] = a[p][j]; a[p][j] = t; }
        }
        for (int i = 1; i < j; ++i)              /* unit-lower trsv (dot of length i) */
            a[i][j] = a[i][j] - a[i][0] * a[0][j];
        if (j > 0)                               /* gemv_n: b[j:] -= A[j:, :j] b[:j] */
            for (int i = j; i < 3; ++i) {
                REAL t = a[i][0] * a[0][j];
                for (int k = 1; k < j; ++k) t = FMA(a[i][k], a[k][j], t);
                a[i][j] = a[i][j] - t;
            }
        int jp = j;                              /* idamax: first max |.| */
        REAL best = FABS(a[j][j]);
        for (int i = j + 1; i < 3; ++i)
            if (FABS(a[i][j]) > best) { best = FABS(a[i][j]); jp = i; }
        piv[j] = jp;
        const REAL r = (REAL)1 / a[jp][j];
        if (jp != j)
            for (int c = 0; c <= j; ++c) { REAL t = a[j][c]; a[j][c] = a[jp][c]; a[jp][c] = t; }
        for (int i = j + 1; i < 3; ++i) a[i][j] = a[i][j] * r;
    }
    /* getrs: B = P I, then L (unit) forward, U backward (inverted diagonal) */
    REAL B[3][3];
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) B[i][k] = (i == k) ? (REAL)1 : (REAL)0;
    for (int j = 0; j < 3; ++j) {
        const int p = piv[j];
        if (p != j)
            for (int k = 0; k < 3; ++k) { REAL t = B[j][k]; B[j][k] = B[p][k]; B[p][k] = t; }
    }
    for (int col = 0; col < 3; ++col) {
        REAL b[3] = {B[0][col], B[1][col], B[2][col]};
        for (int i = 0; i < 3; ++i)
            for (int k = 0; k < i; ++k) b[i] = FMA(-b[k], a[i][k], b[i]);
        b[2] = b[2] * ((REAL)1 / a[2][2]);
        b[0] = b[0] - a[0][2] * b[2];
        b[1] = b[1] - a[1][2] * b[2];
        b[1] = b[1] * ((REAL)1 / a[1][1]);
        b[0] = FMA(-b[1], a[0][1], b[0]);
        b[0] = b[0] * ((REAL)1 / a[0][0]);
        for (int i = 0; i < 3; ++i) Ai[3 * i + col] = b[i];
    }
}

/* ---------------- reference functions ----------------------------------- */
/* compute_inertia_tensor_world, collision.py:51-53:
 *   R.from_quat(q[[1,2,3,0]]).as_matrix() @ diag(I) @ R.T               */
static void FN(rbo_inertia_world)(const REAL I[3], const REAL q[4], REAL Iw[9]) {
    REAL x = q[1], y = q[2], z = q[3], w = q[0];
    const REAL n = SQRT(((x * x + y * y) + z * z) + w * w);    /* SciPy normalise */
    x = x / n; y = y / n; z = z / n; w = w / n;
    const REAL x2 = x * x, y2 = y * y, z2 = z * z, w2 = w * w;
    const REAL xy = x * y, zw = z * w, xz = x * z, yw = y * w, yz = y * z, xw = x * w;
    REAL R[9];
    R[0] = ((x2 - y2) - z2) + w2;   R[1] = 2 * (xy - zw);          R[2] = 2 * (xz + yw);
    R[3] = 2 * (xy + zw);           R[4] = ((-x2 + y2) - z2) + w2; R[5] = 2 * (yz - xw);
    R[6] = 2 * (xz - yw);           R[7] = 2 * (yz + xw);          R[8] = ((-x2 - y2) + z2) + w2;
    const REAL D[9] = {I[0], 0, 0, 0, I[1], 0, 0, 0, I[2]};
    REAL M[9];
    FN(np_gemm3)(R, D, 0, M);
    FN(np_gemm3)(M, R, 1, Iw);
}

/* compute_collision_impulse_friction, collision.py:7-48.  Returns 1 when the
 * contact is separating (u_rel_n >= 0, :32-33: jn = 0, jt = 0). */
static int FN(rbo_impulse)(REAL m, const REAL v[3], const REAL w[3], const REAL r[3],
                           const REAL n[3], REAL e, REAL mu, REAL *jn_out, REAL jt[3]) {
    REAL c[3], u[3], ut[3];
    FN(np_cross)(w, r, c);                                   /* :26 */
    for (int k = 0; k < 3; ++k) u[k] = v[k] + c[k];
    const REAL un = FN(np_dot3)(u, n);                       /* :28 */
    for (int k = 0; k < 3; ++k) ut[k] = u[k] - un * n[k];    /* :29 */
    jt[0] = jt[1] = jt[2] = 0;
    if (un >= 0) { *jn_out = 0; return 1; }                  /* :32-33 */
    const REAL kk = ((REAL)1 / m) + ((REAL)1 / (REAL)18);    /* :36 */
    const REAL jn = (-((REAL)1 + e) * un) / kk;              /* :39 */
    const REAL nut = FN(np_norm3)(ut);
    if (nut > (REAL)1e-6) {                                  /* :43 */
        const REAL mf = mu * FABS(jn);                       /* :44 */
        const REAL s = -((nut < mf) ? nut : mf);             /* :45 min(mf, |ut|) */
        for (int k = 0; k < 3; ++k) jt[k] = s * (ut[k] / nut);
    }
    *jn_out = jn;
    return 0;
}

/* apply_impulse_friction, physics_utils.py:25-49 */
static void FN(rbo_apply)(REAL v[3], REAL w[3], REAL m, const REAL invI[9], const REAL r[3],
                          const REAL n[3], REAL jn, const REAL jt[3]) {
    REAL P[3], cr[3], dw[3];
    for (int k = 0; k < 3; ++k) P[k] = jn * n[k] + jt[k];    /* :42-45 */
    FN(np_cross)(r, P, cr);                                  /* :46-47 */
    FN(np_matvec3)(invI, cr, dw);
    for (int k = 0; k < 3; ++k) { v[k] = v[k] + P[k] / m; w[k] = w[k] + dw[k]; }
}

/* KAT entry: in[24] = m,e,mu,v3,w3,r3,n3,Iw9 -> out[10] = jn,jt3,v'3,w'3 */
int FN(rbo_kat_impulse)(int64_t n, const double *in, double *out) {
    for (int64_t c = 0; c < n; ++c) {
        const double *p = in + 24 * c;
        REAL m = (REAL)p[0], e = (REAL)p[1], mu = (REAL)p[2];
        REAL v[3], w[3], r[3], nn[3], Iw[9], invI[9], jt[3], jn;
        for (int k = 0; k < 3; ++k) {
            v[k] = (REAL)p[3 + k]; w[k] = (REAL)p[6 + k];
            r[k] = (REAL)p[9 + k]; nn[k] = (REAL)p[12 + k];
        }
        for (int k = 0; k < 9; ++k) Iw[k] = (REAL)p[15 + k];
        FN(np_inv3)(Iw, invI);
        FN(rbo_impulse)(m, v, w, r, nn, e, mu, &jn, jt);
        FN(rbo_apply)(v, w, m, invI, r, nn, jn, jt);           /* always applied, as the reference */
        double *o = out + 10 * c;
        o[0] = jn;
        for (int k = 0; k < 3; ++k) { o[1 + k] = jt[k]; o[4 + k] = v[k]; o[7 + k] = w[k]; }
    }
    return 0;
}

/* KAT entry: in[7] = I3, q4 (wxyz) -> out[18] = Iw9, inv(Iw)9 */
int FN(rbo_kat_inertia)(int64_t n, const double *in, double *out) {
    for (int64_t c = 0; c < n; ++c) {
        const double *p = in + 7 * c;
        REAL I[3] = {(REAL)p[0], (REAL)p[1], (REAL)p[2]};
        REAL q[4] = {(REAL)p[3], (REAL)p[4], (REAL)p[5], (REAL)p[6]};
        REAL Iw[9], Ii[9];
        FN(rbo_inertia_world)(I, q, Iw);
        FN(np_inv3)(Iw, Ii);
        for (int k = 0; k < 9; ++k) { out[18 * c + k] = Iw[k]; out[18 * c + 9 + k] = Ii[k]; }
    }
    return 0;
}

/* ---------------- MuJoCo restatements (plain arithmetic) ----------------- */
static inline REAL FN(mj_dot3)(const REAL a[3], const REAL b[3]) {
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
/* mju_mulQuat (w-first Hamilton product) */
static inline void FN(mj_mulquat)(const REAL a[4], const REAL b[4], REAL r[4]) {
    r[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    r[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    r[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
    r[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
}
/* mj_kinematics of a free joint: xquat = mju_normalize4(qpos quat), then
 * xmat = mju_quat2Mat(xquat) */
static void FN(mj_body_mat)(const REAL qin[4], REAL M[9]) {
    REAL q[4] = {qin[0], qin[1], qin[2], qin[3]};
    const REAL nrm = SQRT(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    if (nrm < (REAL)1e-15) { q[0] = 1; q[1] = q[2] = q[3] = 0; }
    else if (FABS(nrm - (REAL)1) > (REAL)1e-15) {
        const REAL inv = (REAL)1 / nrm;
        for (int k = 0; k < 4; ++k) q[k] = q[k] * inv;
    }
    if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) {
        for (int k = 0; k < 9; ++k) M[k] = (k % 4 == 0) ? (REAL)1 : (REAL)0;
        return;
    }
    const REAL q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
    const REAL q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
    const REAL q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
    M[0] = q00 + q11 - q22 - q33;
    M[4] = q00 - q11 + q22 - q33;
    M[8] = q00 - q11 - q22 + q33;
    M[1] = 2 * (q12 - q03);
    M[2] = 2 * (q13 + q02);
    M[3] = 2 * (q12 + q03);
    M[5] = 2 * (q23 - q01);
    M[6] = 2 * (q13 - q02);
    M[7] = 2 * (q23 + q01);
}

typedef struct {
    int32_t partner;   /* body id, or -1 - plane */
    int32_t kind;      /* RB_CK_* */
    int32_t self_g1;   /* the body being solved is geom1 (ORIENTED flips the normal) */
    REAL dist;
    REAL pos[3];
    REAL frame[3];     /* MuJoCo contact normal, geom1 -> geom2 */
} FN(rbo_contact);

/* mjc_PlaneSphere (plane = geom1) */
static int FN(plane_sphere)(const REAL pn[3], const REAL pp[3], const REAL c[3], REAL rad,
                            FN(rbo_contact) *con) {
    REAL tmp[3] = {c[0] - pp[0], c[1] - pp[1], c[2] - pp[2]};
    const REAL cdist = FN(mj_dot3)(tmp, pn);
    if (cdist > (REAL)0 + rad) return 0;
    con->dist = cdist - rad;
    const REAL s = -con->dist / 2 - rad;
    for (int k = 0; k < 3; ++k) { con->pos[k] = c[k] + pn[k] * s; con->frame[k] = pn[k]; }
    con->kind = RB_CK_PLANE_SPHERE;
    return 1;
}

/* mjc_PlaneBox (plane = geom1): corners in bit order, at most 4 contacts */
static int FN(plane_box)(const REAL pn[3], const REAL pp[3], const REAL c[3], const REAL M[9],
                         const REAL h[3], FN(rbo_contact) *con) {
    REAL dif[3] = {c[0] - pp[0], c[1] - pp[1], c[2] - pp[2]};
    const REAL dist = FN(mj_dot3)(dif, pn);
    int cnt = 0;
    for (int i = 0; i < 8; ++i) {
        const REAL vec[3] = {(i & 1) ? h[0] : -h[0], (i & 2) ? h[1] : -h[1], (i & 4) ? h[2] : -h[2]};
        REAL corner[3];
        for (int k = 0; k < 3; ++k)
            corner[k] = M[3 * k] * vec[0] + M[3 * k + 1] * vec[1] + M[3 * k + 2] * vec[2];
        const REAL ldist = FN(mj_dot3)(pn, corner);
        if (dist + ldist > (REAL)0 || ldist > (REAL)0) continue;
        FN(rbo_contact) *cc = con + cnt;
        cc->dist = dist + ldist;
        const REAL s = -cc->dist / 2;
        for (int k = 0; k < 3; ++k) {
            corner[k] = corner[k] + c[k];
            cc->pos[k] = corner[k] + pn[k] * s;
            cc->frame[k] = pn[k];
        }
        cc->kind = RB_CK_PLANE_BOX0 + i;
        if (++cnt >= 4) break;
    }
    return cnt;
}

/* mjc_SphereSphere: geom1 = lower body id */
static int FN(sphere_sphere)(const REAL c1[3], REAL r1, const REAL c2[3], REAL r2,
                             FN(rbo_contact) *con) {
    REAL dif[3] = {c1[0] - c2[0], c1[1] - c2[1], c1[2] - c2[2]};
    const REAL cdist = SQRT(FN(mj_dot3)(dif, dif));
    if (cdist > ((REAL)0 + r1) + r2) return 0;
    con->dist = (cdist - r1) - r2;
    REAL f[3] = {c2[0] - c1[0], c2[1] - c1[1], c2[2] - c1[2]};
    const REAL len = SQRT(FN(mj_dot3)(f, f));                  /* mju_normalize3 */
    if (len < (REAL)1e-15) { f[0] = 1; f[1] = 0; f[2] = 0; }
    else { const REAL inv = (REAL)1 / len; for (int k = 0; k < 3; ++k) f[k] = f[k] * inv; }
    const REAL s = r1 + con->dist / 2;
    for (int k = 0; k < 3; ++k) { con->pos[k] = f[k] * s + c1[k]; con->frame[k] = f[k]; }
    con->kind = RB_CK_SPHERE_SPHERE;
    return 1;
}

/* ---------------- box pairs ---------------------------
 * MuJoCo's mjc_SphereBox and mjc_BoxBox are third-party C that is neither
 * installed nor vendored here, so these are THIS PROJECT'S DEFINITIONS,
 * following the published structure of those primitives (margin 0):
 *   sphere-box: the sphere centre in the box frame is clamped to the box;
 *     outside: normal = clamped - centre (sphere -> box), dist = |.| - r,
 *     pos = midpoint of the clamped point and the sphere's deepest point;
 *     centre inside: the nearest face (faces +x, -x, +y, -y, +z, -z,
 *     first minimum), dist = -(face distance + r).  Sphere = geom1.
 *   box-box: separating-axis test over the 15 axes (A faces, B faces, the 9
 *     edge crosses; an edge axis wins only if 1.05 x its separation beats
 *     the best face axis), normal oriented geom1 -> geom2.  Face axis: the
 *     incident face of the other box (most anti-parallel normal) is clipped
 *     against the reference face rectangle (Sutherland-Hodgman, planes
 *     +a1, -a1, +a2, -a2); clipped points below the reference face are
 *     contacts (at most 4: the 4 deepest, kept in polygon order), pos
 *     halfway between the faces.  Edge axis: one contact at the midpoint of
 *     the closest points of the two supporting edges, dist = the separation.
 * Parity against MuJoCo itself is UNPINNED; the HIP path (csrc/rb_boxes.hpp)
 * must match these bit for bit. */
static void FN(mat_col)(const REAL M[9], int k, REAL u[3]) { u[0] = M[k]; u[1] = M[3 + k]; u[2] = M[6 + k]; }
static inline REAL FN(clampv)(REAL x, REAL lo, REAL hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* sphere (c1, r1) = geom1, box (c2, M2, h2) = geom2 */
static int FN(sphere_box)(const REAL c1[3], REAL r1, const REAL c2[3], const REAL M2[9], const REAL h2[3],
                          FN(rbo_contact) *con) {
    REAL tmp[3], center[3], clamped[3], nearest[3], pos[3], nrm[3];
    for (int k = 0; k < 3; ++k) tmp[k] = c1[k] - c2[k];
    for (int k = 0; k < 3; ++k) center[k] = M2[k] * tmp[0] + M2[3 + k] * tmp[1] + M2[6 + k] * tmp[2];
    for (int k = 0; k < 3; ++k) clamped[k] = FN(clampv)(center[k], -h2[k], h2[k]);
    for (int k = 0; k < 3; ++k) nearest[k] = clamped[k] - center[k];
    const REAL dist = SQRT(FN(mj_dot3)(nearest, nearest));
    if (dist - r1 > (REAL)0) return 0;
    REAL cd;
    if (dist <= (REAL)1e-15) {
        REAL closest = (REAL)2 * ((h2[0] + h2[1]) + h2[2]);
        int kf = 0;
        for (int i = 0; i < 6; ++i) {
            const int a = i / 2;
            const REAL df = (i % 2 == 0) ? h2[a] - center[a] : h2[a] + center[a];
            if (df < closest) { closest = df; kf = i; }
        }
        const int a = kf / 2;
        const REAL s = (kf % 2 == 0) ? (REAL)1 : (REAL)-1;
        for (int k = 0; k < 3; ++k) { nrm[k] = (REAL)0; pos[k] = center[k]; }
        nrm[a] = -s;
        pos[a] = center[a] + s * ((closest - r1) / (REAL)2);
        cd = -closest - r1;
    } else {
        const REAL inv = (REAL)1 / dist;
        for (int k = 0; k < 3; ++k) nrm[k] = nearest[k] * inv;
        for (int k = 0; k < 3; ++k) pos[k] = (clamped[k] + (center[k] + nrm[k] * r1)) * (REAL)0.5;
        cd = dist - r1;
    }
    for (int k = 0; k < 3; ++k) {
        con->pos[k] = (M2[3 * k] * pos[0] + M2[3 * k + 1] * pos[1] + M2[3 * k + 2] * pos[2]) + c2[k];
        con->frame[k] = M2[3 * k] * nrm[0] + M2[3 * k + 1] * nrm[1] + M2[3 * k + 2] * nrm[2];
    }
    con->dist = cd;
    con->kind = RB_CK_SPHERE_BOX;
    return 1;
}

/* box A (pa, Ma, ha) = geom1, box B = geom2; up to 4 contacts into con */
static int FN(box_box)(const REAL pa[3], const REAL Ma[9], const REAL ha[3], const REAL pb[3], const REAL Mb[9],
                       const REAL hb[3], FN(rbo_contact) *con) {
    REAL ua[3][3], ub[3][3], d[3], R[3][3], AR[3][3], da[3], db[3];
    for (int i = 0; i < 3; ++i) { FN(mat_col)(Ma, i, ua[i]); FN(mat_col)(Mb, i, ub[i]); }
    for (int k = 0; k < 3; ++k) d[k] = pb[k] - pa[k];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) { R[i][j] = FN(mj_dot3)(ua[i], ub[j]); AR[i][j] = FABS(R[i][j]); }
    for (int i = 0; i < 3; ++i) { da[i] = FN(mj_dot3)(d, ua[i]); db[i] = FN(mj_dot3)(d, ub[i]); }
    REAL best = (REAL)0, L[3] = {0, 0, 0}, dL = 0;
    int bk = -1;
    for (int i = 0; i < 3; ++i) {
        const REAL s = FABS(da[i]) - (ha[i] + ((hb[0] * AR[i][0] + hb[1] * AR[i][1]) + hb[2] * AR[i][2]));
        if (s > (REAL)0) return 0;
        if (bk < 0 || s > best) { best = s; bk = i; }
    }
    for (int j = 0; j < 3; ++j) {
        const REAL s = FABS(db[j]) - (((ha[0] * AR[0][j] + ha[1] * AR[1][j]) + ha[2] * AR[2][j]) + hb[j]);
        if (s > (REAL)0) return 0;
        if (s > best) { best = s; bk = 3 + j; }
    }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            const REAL *a = ua[i], *b = ub[j];
            REAL c[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
            const REAL len = SQRT(FN(mj_dot3)(c, c));
            if (len < (REAL)1e-6) continue;                       /* parallel edges */
            const REAL inv = (REAL)1 / len;
            for (int k = 0; k < 3; ++k) c[k] = c[k] * inv;
            const REAL pA = (ha[0] * FABS(FN(mj_dot3)(ua[0], c)) + ha[1] * FABS(FN(mj_dot3)(ua[1], c))) +
                            ha[2] * FABS(FN(mj_dot3)(ua[2], c));
            const REAL pB = (hb[0] * FABS(FN(mj_dot3)(ub[0], c)) + hb[1] * FABS(FN(mj_dot3)(ub[1], c))) +
                            hb[2] * FABS(FN(mj_dot3)(ub[2], c));
            const REAL dc = FN(mj_dot3)(d, c);
            const REAL s = FABS(dc) - (pA + pB);
            if (s > (REAL)0) return 0;
            if (s * (REAL)1.05 > best) { best = s; bk = 6 + 3 * i + j; L[0] = c[0]; L[1] = c[1]; L[2] = c[2]; dL = dc; }
        }
    if (bk < 3) { for (int k = 0; k < 3; ++k) L[k] = ua[bk][k]; dL = da[bk]; }
    else if (bk < 6) { for (int k = 0; k < 3; ++k) L[k] = ub[bk - 3][k]; dL = db[bk - 3]; }
    REAL n[3];
    for (int k = 0; k < 3; ++k) n[k] = dL < (REAL)0 ? -L[k] : L[k];

    if (bk >= 6) {                                                /* edge - edge */
        const int i = (bk - 6) / 3, j = (bk - 6) % 3;
        REAL qa[3] = {pa[0], pa[1], pa[2]}, qb[3] = {pb[0], pb[1], pb[2]}, r[3];
        for (int k = 0; k < 3; ++k) {
            if (k == i) continue;
            const REAL sg = FN(mj_dot3)(ua[k], n) > (REAL)0 ? ha[k] : -ha[k];
            for (int c = 0; c < 3; ++c) qa[c] = qa[c] + ua[k][c] * sg;
        }
        for (int k = 0; k < 3; ++k) {
            if (k == j) continue;
            const REAL sg = FN(mj_dot3)(ub[k], n) > (REAL)0 ? -hb[k] : hb[k];
            for (int c = 0; c < 3; ++c) qb[c] = qb[c] + ub[k][c] * sg;
        }
        for (int k = 0; k < 3; ++k) r[k] = qb[k] - qa[k];
        const REAL a = R[i][j], e = FN(mj_dot3)(ua[i], r), f = FN(mj_dot3)(ub[j], r);
        const REAL den = (REAL)1 - a * a;
        const REAL s = FN(clampv)((e - a * f) / den, -ha[i], ha[i]);
        const REAL t = FN(clampv)((a * e - f) / den, -hb[j], hb[j]);
        for (int k = 0; k < 3; ++k) {
            con->pos[k] = ((qa[k] + ua[i][k] * s) + (qb[k] + ub[j][k] * t)) * (REAL)0.5;
            con->frame[k] = n[k];
        }
        con->dist = best;
        con->kind = RB_CK_BOX_EDGE;
        return 1;
    }

    /* face: reference box (the axis's owner), incident box (the other) */
    const int refa = bk < 3, ra = refa ? bk : bk - 3;
    const REAL *pr = refa ? pa : pb, *pi = refa ? pb : pa, *hr = refa ? ha : hb, *hi = refa ? hb : ha;
    REAL (*ur)[3] = refa ? ua : ub, (*ui)[3] = refa ? ub : ua;
    REAL nr[3], cdot[3], cinc[3], e1[3], e2[3], cref[3];
    for (int k = 0; k < 3; ++k) nr[k] = refa ? n[k] : -n[k];    /* reference face normal, toward the incident box */
    int kk = 0;
    REAL cb = (REAL)-1;
    for (int k = 0; k < 3; ++k) {
        cdot[k] = FN(mj_dot3)(ui[k], nr);
        if (FABS(cdot[k]) > cb) { cb = FABS(cdot[k]); kk = k; }
    }
    const REAL sg = cdot[kk] > (REAL)0 ? (REAL)-1 : (REAL)1;
    const int b1 = kk == 0 ? 1 : 0, b2 = kk == 2 ? 1 : 2;
    const int a1 = ra == 0 ? 1 : 0, a2 = ra == 2 ? 1 : 2;
    for (int k = 0; k < 3; ++k) {
        cinc[k] = pi[k] + ui[kk][k] * (sg * hi[kk]);
        e1[k] = ui[b1][k] * hi[b1];
        e2[k] = ui[b2][k] * hi[b2];
        cref[k] = pr[k] + nr[k] * hr[ra];
    }
    REAL P[8][3], Q[8][3];
    int np = 4;
    for (int v = 0; v < 4; ++v) {                                 /* (+,+) (-,+) (-,-) (+,-) */
        REAL vert[3], rel[3];
        for (int k = 0; k < 3; ++k) {
            vert[k] = (v == 0 || v == 3) ? cinc[k] + e1[k] : cinc[k] - e1[k];
            vert[k] = (v < 2) ? vert[k] + e2[k] : vert[k] - e2[k];
            rel[k] = vert[k] - cref[k];
        }
        P[v][0] = FN(mj_dot3)(rel, ur[a1]);
        P[v][1] = FN(mj_dot3)(rel, ur[a2]);
        P[v][2] = FN(mj_dot3)(rel, nr);
    }
    for (int pl = 0; pl < 4 && np > 0; ++pl) {
        const int c = pl < 2 ? 0 : 1, neg = pl & 1;
        const REAL w = pl < 2 ? hr[a1] : hr[a2];
        int nq = 0;
        for (int t = 0; t < np; ++t) {
            const REAL *cur = P[t], *prv = P[(t + np - 1) % np];
            const REAL fc = (neg ? -cur[c] : cur[c]) - w;
            const REAL fp = (neg ? -prv[c] : prv[c]) - w;
            const int ins = fc <= (REAL)0, pins = fp <= (REAL)0;
            if (ins != pins && nq < 8) {                          /* the edge crosses the plane */
                const REAL tt = fp / (fp - fc);
                for (int k = 0; k < 3; ++k) Q[nq][k] = prv[k] + (cur[k] - prv[k]) * tt;
                ++nq;
            }
            if (ins && nq < 8) { for (int k = 0; k < 3; ++k) Q[nq][k] = cur[k]; ++nq; }
        }
        for (int t = 0; t < nq; ++t) for (int k = 0; k < 3; ++k) P[t][k] = Q[t][k];
        np = nq;
    }
    unsigned keep = 0;
    int nk = 0;
    for (int t = 0; t < np; ++t) if (P[t][2] <= (REAL)0) { keep |= 1u << t; ++nk; }
    if (nk > 4) {                                                 /* the 4 deepest */
        unsigned pick = 0;
        for (int r = 0; r < 4; ++r) {
            int bt = -1;
            for (int t = 0; t < np; ++t)
                if (((keep & ~pick) >> t) & 1u) if (bt < 0 || P[t][2] < P[bt][2]) bt = t;
            pick |= 1u << bt;
        }
        keep = pick;
    }
    int m = 0;
    for (int t = 0; t < np; ++t) {
        if (!((keep >> t) & 1u)) continue;
        const REAL x = P[t][0], y = P[t][1], z = P[t][2], s = -z / (REAL)2;
        for (int k = 0; k < 3; ++k) {
            const REAL wp = ((cref[k] + ur[a1][k] * x) + ur[a2][k] * y) + nr[k] * z;
            con[m].pos[k] = wp + nr[k] * s;
            con[m].frame[k] = n[k];
        }
        con[m].dist = z;
        con[m].kind = RB_CK_BOX_BOX0 + m;
        ++m;
    }
    return m;
}

/* The contacts of the pair (i, j) in MuJoCo's geom order — spheres by id,
 * sphere before box, boxes by id — into con (at most 4); self_g1 marks
 * whether body i is geom1. */
static int FN(pair_contacts)(const rb_scene_desc *d, const REAL *pos, const REAL *quat, int64_t i, int64_t j,
                             FN(rbo_contact) *con) {
    const int si = d->kind[i] == RB_BODY_SPHERE, sj = d->kind[j] == RB_BODY_SPHERE;
    int64_t g1, g2;
    if (si != sj) { g1 = si ? i : j; g2 = si ? j : i; }
    else { g1 = i < j ? i : j; g2 = i < j ? j : i; }
    int nc;
    if (si && sj) {
        nc = FN(sphere_sphere)(pos + 3 * g1, (REAL)d->size[3 * g1], pos + 3 * g2, (REAL)d->size[3 * g2], con);
    } else if (si != sj) {
        REAL M[9], h[3] = {(REAL)d->size[3 * g2], (REAL)d->size[3 * g2 + 1], (REAL)d->size[3 * g2 + 2]};
        FN(mj_body_mat)(quat + 4 * g2, M);
        nc = FN(sphere_box)(pos + 3 * g1, (REAL)d->size[3 * g1], pos + 3 * g2, M, h, con);
    } else {
        REAL M1[9], M2[9];
        REAL h1[3] = {(REAL)d->size[3 * g1], (REAL)d->size[3 * g1 + 1], (REAL)d->size[3 * g1 + 2]};
        REAL h2[3] = {(REAL)d->size[3 * g2], (REAL)d->size[3 * g2 + 1], (REAL)d->size[3 * g2 + 2]};
        FN(mj_body_mat)(quat + 4 * g1, M1);
        FN(mj_body_mat)(quat + 4 * g2, M2);
        nc = FN(box_box)(pos + 3 * g1, M1, h1, pos + 3 * g2, M2, h2, con);
    }
    for (int t = 0; t < nc; ++t) { con[t].partner = (int32_t)j; con[t].self_g1 = g1 == i; }
    return nc;
}

/* KAT entry: in[22] = kind1, kind2, c1[3], q1[4], s1[3], c2[3], q2[4], s2[3]
 * (body 1 has the lower id) -> out[33] = count, then per contact dist,
 * pos[3], frame[3], kind (from body 1's side: frame as generated). */
int FN(rbo_kat_narrow)(int64_t n, const double *in, double *out) {
    for (int64_t c = 0; c < n; ++c) {
        const double *a = in + 22 * c;
        int32_t kinds[2] = {(int32_t)a[0], (int32_t)a[1]};
        double sz[6] = {a[9], a[10], a[11], a[19], a[20], a[21]};
        rb_scene_desc dd;
        memset(&dd, 0, sizeof dd);
        dd.n_bodies = 2;
        dd.kind = kinds;
        dd.size = sz;
        REAL pos[6] = {(REAL)a[2], (REAL)a[3], (REAL)a[4], (REAL)a[12], (REAL)a[13], (REAL)a[14]};
        REAL quat[8] = {(REAL)a[5], (REAL)a[6], (REAL)a[7], (REAL)a[8], (REAL)a[15], (REAL)a[16], (REAL)a[17], (REAL)a[18]};
        FN(rbo_contact) con[4];
        const int nc = FN(pair_contacts)(&dd, pos, quat, 0, 1, con);
        double *o = out + 33 * c;
        for (int k = 0; k < 33; ++k) o[k] = 0;
        o[0] = nc;
        for (int t = 0; t < nc; ++t) {
            double *r = o + 1 + 8 * t;
            r[0] = (double)con[t].dist;
            for (int k = 0; k < 3; ++k) { r[1 + k] = (double)con[t].pos[k]; r[4 + k] = (double)con[t].frame[k]; }
            r[7] = con[t].kind;
        }
    }
    return 0;
}

/* ---------------- broadphase (oracle: exact cell keys, sorted) ------------ */
typedef struct { int64_t key; int64_t id; } FN(cellrec);
static int FN(cell_cmp)(const void *a, const void *b) {
    const FN(cellrec) *x = a, *y = b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->id < y->id ? -1 : (x->id > y->id);
}
static inline int64_t FN(cell_key)(int64_t ix, int64_t iy, int64_t iz) {
    return ((ix + (1 << 20)) << 42) | ((iy + (1 << 20)) << 21) | (iz + (1 << 20));
}

static REAL FN(bound_radius)(const rb_scene_desc *d, int64_t i) {
    const double *s = d->size + 3 * i;
    if (d->kind[i] == RB_BODY_SPHERE) return (REAL)s[0];
    return SQRT((REAL)(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]));
}

/* Per-body canonical contact lists for positions pos[N][3] / quats: body i's
 * contacts are cons[i * stride + t], t < counts[i] (stride = 4 * n_planes +
 * max_partners bounds them).  Bodies are independent after the cell sort
 * (OpenMP over bodies when built with -fopenmp; results do not depend on the
 * thread count). */
static int FN(gen_contacts)(const rb_scene_desc *d, const REAL *pos, const REAL *quat,
                            int32_t *counts, FN(rbo_contact) *cons, int64_t stride) {
    const int64_t N = d->n_bodies;
    const int maxp = d->max_partners > 0 ? d->max_partners : 16;
    REAL rmax = 0;
    for (int64_t i = 0; i < N; ++i) { REAL b = FN(bound_radius)(d, i); if (b > rmax) rmax = b; }
    const REAL cs = rmax > 0 ? (REAL)2 * rmax * (REAL)1.001 : (REAL)1;
    FN(cellrec) *cells = (FN(cellrec) *)malloc(sizeof(FN(cellrec)) * (size_t)(N > 0 ? N : 1));
    int64_t *ix = (int64_t *)malloc(sizeof(int64_t) * 3 * (size_t)(N > 0 ? N : 1));
    if (!cells || !ix) { free(cells); free(ix); return RB_ENOMEM; }
    int rc = RB_OK;
    for (int64_t i = 0; i < N; ++i) {
        for (int k = 0; k < 3; ++k) {
            const REAL p = pos[3 * i + k];
            if (!(p == p) || FABS(p) > cs * (REAL)1000000) { rc = RB_EDOM; goto done; }
            ix[3 * i + k] = (int64_t)floor((double)(p / cs));
        }
        cells[i].key = FN(cell_key)(ix[3 * i], ix[3 * i + 1], ix[3 * i + 2]);
        cells[i].id = i;
    }
    qsort(cells, (size_t)N, sizeof(FN(cellrec)), FN(cell_cmp));
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t i = 0; i < N; ++i) {
        int64_t plist[33];
        int64_t off = i * stride;
        int32_t cnt = 0;
        int brc = RB_OK;
        const REAL *ci = pos + 3 * i;
        /* planes first, plane order */
        for (int p = 0; p < d->n_planes; ++p) {
            REAL pn[3], pp[3];
            for (int k = 0; k < 3; ++k) { pn[k] = (REAL)d->planes[6 * p + k]; pp[k] = (REAL)d->planes[6 * p + 3 + k]; }
            FN(rbo_contact) tmp[4];
            int nc;
            if (d->kind[i] == RB_BODY_SPHERE) nc = FN(plane_sphere)(pn, pp, ci, (REAL)d->size[3 * i], tmp);
            else {
                REAL M[9], h[3] = {(REAL)d->size[3 * i], (REAL)d->size[3 * i + 1], (REAL)d->size[3 * i + 2]};
                FN(mj_body_mat)(quat + 4 * i, M);
                nc = FN(plane_box)(pn, pp, ci, M, h, tmp);
            }
            for (int t = 0; t < nc; ++t) {
                tmp[t].partner = -1 - p;
                tmp[t].self_g1 = 0;
                cons[off++] = tmp[t];
                ++cnt;
            }
        }
        /* sphere partners: 27 neighbour cells, exact test, ascending id */
        int np_ = 0;
        for (int dx = -1; dx <= 1; ++dx)
            for (int dy = -1; dy <= 1; ++dy)
                for (int dz = -1; dz <= 1; ++dz) {
                    FN(cellrec) probe = {FN(cell_key)(ix[3 * i] + dx, ix[3 * i + 1] + dy, ix[3 * i + 2] + dz), -1};
                    /* lower bound */
                    int64_t lo = 0, hi = N;
                    while (lo < hi) {
                        int64_t mid = (lo + hi) / 2;
                        if (FN(cell_cmp)(&cells[mid], &probe) < 0) lo = mid + 1; else hi = mid;
                    }
                    for (int64_t t = lo; t < N && cells[t].key == probe.key && !brc; ++t) {
                        const int64_t j = cells[t].id;
                        if (j == i) continue;
                        const REAL *cj = pos + 3 * j;
                        if (d->kind[i] != RB_BODY_SPHERE || d->kind[j] != RB_BODY_SPHERE) {
                            /* box-involved pair: a partner when the bounding spheres overlap
                             * (the narrowphase may then find no contact) */
                            REAL dd[3] = {ci[0] - cj[0], ci[1] - cj[1], ci[2] - cj[2]};
                            const REAL bi = FN(bound_radius)(d, i), bj = FN(bound_radius)(d, j);
                            if (!(SQRT(FN(mj_dot3)(dd, dd)) <= bi + bj)) continue;
                        } else {
                            const int64_t g1 = i < j ? i : j, g2 = i < j ? j : i;
                            FN(rbo_contact) con;
                            if (!FN(sphere_sphere)(pos + 3 * g1, (REAL)d->size[3 * g1], pos + 3 * g2,
                                                   (REAL)d->size[3 * g2], &con)) continue;
                        }
                        if (np_ >= maxp) { brc = RB_EOVERFLOW; break; }
                        /* insertion into ascending id order */
                        int s = np_++;
                        while (s > 0 && plist[s - 1] > j) { plist[s] = plist[s - 1]; --s; }
                        plist[s] = j;
                    }
                }
        for (int s = 0; s < np_; ++s) {
            FN(rbo_contact) con[4];
            const int nc = FN(pair_contacts)(d, pos, quat, i, plist[s], con);
            for (int t = 0; t < nc; ++t) { cons[off++] = con[t]; ++cnt; }
        }
        counts[i] = cnt;
        if (brc) {
#pragma omp critical
            if (rc == RB_OK) rc = brc;
        }
    }
done:
    free(cells); free(ix);
    return rc;
}

/* contact records per body: 4 per plane, 1 per sphere partner, 4 per
 * partner in scenes with boxes */
static int64_t FN(contact_stride)(const rb_scene_desc *d) {
    const int maxp = d->max_partners > 0 ? d->max_partners : 16;
    int boxes = 0;
    for (int64_t i = 0; i < d->n_bodies && !boxes; ++i) boxes = d->kind[i] != RB_BODY_SPHERE;
    return 4 * (int64_t)d->n_planes + (boxes ? 4 : 1) * (int64_t)maxp;
}

/* ---------------- the step (a8/a9) ------------------------------------ */
/* nsteps reference steps on AoS qpos[N*7] / qvel[N*6] (in place).
 * Follows collision.py:56-102 / time_integeration.py:13-72 per body and
 * multi_sphere_bounce.py:42-92 across bodies (one contact pass per step).
 * Optional: contact list of the last step (CSR over all bodies). */
int FN(rbo_step)(const rb_scene_desc *d, double *qpos, double *qvel, const double *xfrc,
                 int64_t nsteps, double dt_, double e_, double mu_, double thr_,
                 int32_t *out_counts, int32_t *out_partner, int32_t *out_kind, double *out_dist,
                 int64_t out_cap, int64_t *out_total) {
    const int64_t N = d->n_bodies;
    const REAL dt = (REAL)dt_, e = (REAL)e_, mu = (REAL)mu_, thr = (REAL)thr_;
    const int64_t stride = FN(contact_stride)(d);
    REAL *pos = (REAL *)calloc(3 * (size_t)(N + 1), sizeof(REAL));
    REAL *quat = (REAL *)calloc(4 * (size_t)(N + 1), sizeof(REAL));
    REAL *vel = (REAL *)malloc(sizeof(REAL) * 6 * (size_t)(N + 1));
    int32_t *counts = (int32_t *)malloc(sizeof(int32_t) * (size_t)(N + 1));
    FN(rbo_contact) *cons = (FN(rbo_contact) *)malloc(sizeof(FN(rbo_contact)) * (size_t)(N * stride + 1));
    int rc = RB_OK;
    if (!pos || !quat || !vel || !counts || !cons) { rc = RB_ENOMEM; goto out; }
    for (int64_t i = 0; i < N; ++i) {
        for (int k = 0; k < 3; ++k) pos[3 * i + k] = (REAL)qpos[7 * i + k];
        for (int k = 0; k < 4; ++k) quat[4 * i + k] = (REAL)qpos[7 * i + 3 + k];
        for (int k = 0; k < 6; ++k) vel[6 * i + k] = (REAL)qvel[6 * i + k];
    }
    REAL g[3] = {(REAL)d->gravity[0], (REAL)d->gravity[1], (REAL)d->gravity[2]};
    for (int64_t step = 0; step < nsteps; ++step) {
        rc = FN(gen_contacts)(d, pos, quat, counts, cons, stride);   /* mj_forward */
        if (rc) goto out;
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < N; ++i) {
            const REAL m = (REAL)d->mass[i];
            const REAL I[3] = {(REAL)d->inertia[3 * i], (REAL)d->inertia[3 * i + 1], (REAL)d->inertia[3 * i + 2]};
            REAL *x = pos + 3 * i, *q = quat + 4 * i;
            REAL v[3] = {vel[6 * i], vel[6 * i + 1], vel[6 * i + 2]};
            REAL w[3] = {vel[6 * i + 3], vel[6 * i + 4], vel[6 * i + 5]};
            REAL Iw[9], invI[9];
            FN(rbo_inertia_world)(I, q, Iw);                         /* collision.py:62 */
            FN(np_inv3)(Iw, invI);
            for (int k = 0; k < 3; ++k) {                            /* :66-69 */
                const REAL F = xfrc ? (REAL)xfrc[6 * i + k] + m * g[k] : m * g[k];
                v[k] = v[k] + (F / m) * dt;
            }
            if (xfrc) {                                              /* :70 */
                REAL tdt[3], dw[3];
                for (int k = 0; k < 3; ++k) tdt[k] = (REAL)xfrc[6 * i + 3 + k] * dt;
                FN(np_matvec3)(invI, tdt, dw);
                for (int k = 0; k < 3; ++k) w[k] = w[k] + dw[k];
            }
            for (int64_t c = i * stride; c < i * stride + counts[i]; ++c) {  /* :72-88 */
                const FN(rbo_contact) *cc = cons + c;
                if (!(cc->dist < 0)) continue;                       /* :74 (NaN too) */
                if (FABS(cc->dist) < thr) continue;                  /* :79-80 */
                REAL r[3], n[3];
                const int flip = d->normal_convention == RB_NORMAL_ORIENTED && cc->self_g1;
                for (int k = 0; k < 3; ++k) {
                    r[k] = cc->pos[k] - x[k];                        /* :75 */
                    n[k] = flip ? -cc->frame[k] : cc->frame[k];      /* :76 (D8) */
                }
                REAL jn, jt[3];
                if (FN(rbo_impulse)(m, v, w, r, n, e, mu, &jn, jt)) continue;  /* zero impulse */
                FN(rbo_apply)(v, w, m, invI, r, n, jn, jt);
            }
            /* :90-95 integrate (contact generation for every body is done) */
            for (int k = 0; k < 3; ++k) x[k] = x[k] + v[k] * dt;
            const REAL oq[4] = {0, w[0], w[1], w[2]};
            REAL res[4], qn[4];
            FN(mj_mulquat)(oq, q, res);
            for (int k = 0; k < 4; ++k) qn[k] = q[k] + ((REAL)0.5 * res[k]) * dt;
            const REAL nq = FN(np_norm4)(qn);
            for (int k = 0; k < 4; ++k) q[k] = qn[k] / nq;
            for (int k = 0; k < 3; ++k) { vel[6 * i + k] = v[k]; vel[6 * i + 3 + k] = w[k]; }
        }
    }
    for (int64_t i = 0; i < N; ++i) {
        for (int k = 0; k < 3; ++k) qpos[7 * i + k] = (double)pos[3 * i + k];
        for (int k = 0; k < 4; ++k) qpos[7 * i + 3 + k] = (double)quat[4 * i + k];
        for (int k = 0; k < 6; ++k) qvel[6 * i + k] = (double)vel[6 * i + k];
    }
    if (out_counts && nsteps > 0) {
        int64_t t = 0;
        for (int64_t i = 0; i < N; ++i) {
            out_counts[i] = counts[i];
            for (int64_t c = i * stride; c < i * stride + counts[i]; ++c, ++t) {
                if (t < out_cap) {
                    out_partner[t] = cons[c].partner;
                    out_kind[t] = cons[c].kind;
                    out_dist[t] = (double)cons[c].dist;
                }
            }
        }
        if (out_total) *out_total = t;
        if (t > out_cap) rc = RB_EOVERFLOW;
    }
out:
    free(pos); free(quat); free(vel); free(counts); free(cons);
    return rc;
}

/* Contact lists for one state without stepping (CSR, all bodies), with the
 * full records (pos, frame) for golden comparison. */
int FN(rbo_contacts)(const rb_scene_desc *d, const double *qpos, int32_t *out_counts,
                     int32_t *out_partner, int32_t *out_kind, double *out_dist, double *out_pos,
                     double *out_frame, int64_t out_cap, int64_t *out_total) {
    const int64_t N = d->n_bodies;
    const int64_t stride = FN(contact_stride)(d);
    REAL *pos = (REAL *)calloc(3 * (size_t)(N + 1), sizeof(REAL));
    REAL *quat = (REAL *)calloc(4 * (size_t)(N + 1), sizeof(REAL));
    int32_t *counts = (int32_t *)malloc(sizeof(int32_t) * (size_t)(N + 1));
    FN(rbo_contact) *cons = (FN(rbo_contact) *)malloc(sizeof(FN(rbo_contact)) * (size_t)(N * stride + 1));
    int rc = RB_OK;
    if (!pos || !quat || !counts || !cons) { rc = RB_ENOMEM; goto out; }
    for (int64_t i = 0; i < N; ++i) {
        for (int k = 0; k < 3; ++k) pos[3 * i + k] = (REAL)qpos[7 * i + k];
        for (int k = 0; k < 4; ++k) quat[4 * i + k] = (REAL)qpos[7 * i + 3 + k];
    }
    rc = FN(gen_contacts)(d, pos, quat, counts, cons, stride);
    if (rc) goto out;
    int64_t t = 0;
    for (int64_t i = 0; i < N; ++i) {
        out_counts[i] = counts[i];
        for (int64_t c = i * stride; c < i * stride + counts[i]; ++c, ++t) {
            if (t >= out_cap) continue;
            out_partner[t] = cons[c].partner;
            out_kind[t] = cons[c].kind;
            out_dist[t] = (double)cons[c].dist;
            for (int k = 0; k < 3; ++k) {
                out_pos[3 * t + k] = (double)cons[c].pos[k];
                out_frame[3 * t + k] = (double)cons[c].frame[k];
            }
        }
    }
    *out_total = t;
    if (t > out_cap) rc = RB_EOVERFLOW;
out:
    free(pos); free(quat); free(counts); free(cons);
    return rc;
}

/* FN / CAT stay defined: rb_oracle_pairs.h follows and undefines them */
