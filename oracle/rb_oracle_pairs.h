/*
 * rb_oracle_pairs.h — CPU oracle of the reference's second contact law, the
 * symmetric two-ball impulse of src/simulation/ball_collision.py, included
 * twice by rb_oracle.c (REAL=double/float).  TEST INFRASTRUCTURE ONLY (see
 * rb_oracle_impl.h).
 *
 * What it restates (ball_collision.py):
 *   :39-41   compute_inverse_inertia  I_inv = eye(3) / ((2/5) m r^2)
 *   :53-68   compute_collision_impulse (full effective mass, clipped friction)
 *   :73-125  step_with_custom_collisions: gravity v += g dt; ground contact
 *            of each ball against z = 0 when z < r (impulse, then z = r);
 *            ball-ball contact when |p2 - p1| < 2r + tol (impulse from ball
 *            1's side applied +/- to both, positions pushed apart by half the
 *            overlap); x += v dt; the quaternion is never touched.
 * N balls: the reference has exactly two.  The generalisation here is
 * Jacobi over pairs: every pair (a < b) with |p_b - p_a| < r_a + r_b + tol
 * is evaluated from the post-ground state of both balls, and each ball
 * accumulates its pairs' velocity / spin / position deltas in ascending
 * partner id.  For two balls this is the reference step exactly; for more it
 * is this project's definition (parity against this oracle only).
 */

/* ball_collision.py:53-68 */
static void FN(rbo_pair_impulse)(REAL mass, const REAL Iinv[9], const REAL v[3], const REAL w[3],
                                 const REAL r[3], const REAL n[3], REAL e, REAL mu, REAL out[3]) {
    REAL c[3], vc[3], vt[3], rxn[3], a[3], axr[3], td[3] = {0, 0, 0}, rxt[3], b[3], bxr[3];
    FN(np_cross)(w, r, c);
    for (int k = 0; k < 3; ++k) vc[k] = v[k] + c[k];                       /* :54 */
    const REAL vn = FN(np_dot3)(vc, n);                                     /* :55 */
    for (int k = 0; k < 3; ++k) vt[k] = vc[k] - vn * n[k];                 /* :56 */
    const REAL tn = FN(np_norm3)(vt);                                       /* :57 */
    FN(np_cross)(r, n, rxn);
    FN(np_matvec3)(Iinv, rxn, a);
    FN(np_cross)(a, r, axr);
    const REAL dn = ((REAL)1 / mass) + FN(np_dot3)(n, axr);                 /* :59 */
    const REAL jn = (-((REAL)1 + e) * vn) / dn;                             /* :60 */
    if (tn > (REAL)1e-8)                                                    /* :62 */
        for (int k = 0; k < 3; ++k) td[k] = vt[k] / tn;
    FN(np_cross)(r, td, rxt);
    FN(np_matvec3)(Iinv, rxt, b);
    FN(np_cross)(b, r, bxr);
    const REAL dt_ = ((REAL)1 / mass) + FN(np_dot3)(td, bxr);               /* :63-64 */
    const REAL jtu = -tn / dt_;                                             /* :65 */
    const REAL lim = mu * FABS(jn);
    REAL jt = jtu > -lim ? jtu : -lim;                                      /* :66 np.clip */
    jt = jt < lim ? jt : lim;
    for (int k = 0; k < 3; ++k) out[k] = jn * n[k] + jt * td[k];           /* :68 */
}

/* ball_collision.py:39-41: (2/5) m r^2, then eye(3) / I */
static void FN(rbo_ball_iinv)(REAL m, REAL r, REAL Iinv[9]) {
    const REAL I = ((REAL)0.4 * m) * (r * r);
    for (int k = 0; k < 9; ++k) Iinv[k] = (k % 4 == 0) ? (REAL)1 / I : (REAL)0 / I;
}

/* KAT: in[27] = m, e, mu, v3, w3, r3, n3, Iinv9 -> out[3] = impulse */
int FN(rbo_kat_pair_impulse)(int64_t n, const double *in, double *out) {
    for (int64_t c = 0; c < n; ++c) {
        const double *p = in + 27 * c;
        REAL v[3], w[3], r[3], nn[3], Ii[9], o[3];
        for (int k = 0; k < 3; ++k) {
            v[k] = (REAL)p[3 + k]; w[k] = (REAL)p[6 + k]; r[k] = (REAL)p[9 + k]; nn[k] = (REAL)p[12 + k];
        }
        for (int k = 0; k < 9; ++k) Ii[k] = (REAL)p[15 + k];
        FN(rbo_pair_impulse)((REAL)p[0], Ii, v, w, r, nn, (REAL)p[1], (REAL)p[2], o);
        for (int k = 0; k < 3; ++k) out[3 * c + k] = (double)o[k];
    }
    return 0;
}

/* Gravity and ground contact of one ball (ball_collision.py:77-97), in place. */
static void FN(ball_ground)(REAL p[3], REAL v[3], REAL w[3], REAL m, REAL rad, const REAL Iinv[9],
                            const REAL g[3], REAL dt, REAL e, REAL mu, int ground) {
    for (int k = 0; k < 3; ++k) v[k] = v[k] + g[k] * dt;                   /* :78 */
    if (!ground || !(p[2] < rad)) return;                                   /* :90 */
    const REAL nrm[3] = {0, 0, 1};                                          /* :88 */
    REAL cp[3], rr[3], imp[3], cr[3], dw[3];
    for (int k = 0; k < 3; ++k) cp[k] = p[k] - rad * nrm[k];               /* :91 */
    for (int k = 0; k < 3; ++k) rr[k] = cp[k] - p[k];                      /* :92 */
    FN(rbo_pair_impulse)(m, Iinv, v, w, rr, nrm, e, mu, imp);               /* :93-94 */
    FN(np_cross)(rr, imp, cr);
    FN(np_matvec3)(Iinv, cr, dw);
    for (int k = 0; k < 3; ++k) { v[k] = v[k] + imp[k] / m; w[k] = w[k] + dw[k]; }   /* :95-96 */
    p[2] = rad;                                                             /* :97 */
}

/* The pair (a < b) as seen by ball `self` (a or b): velocity, spin and
 * position deltas applied in place (ball_collision.py:100-118). */
static void FN(ball_pair_apply)(int self_is_a, const REAL pa[3], const REAL va[3], const REAL wa[3], REAL ma,
                                const REAL Ia[9], REAL ra, const REAL pb[3], REAL mb, const REAL Ib[9], REAL rb,
                                REAL tol, REAL e, REAL mu, REAL p[3], REAL v[3], REAL w[3]) {
    REAL diff[3], nrm[3], cp[3], r1[3], r2[3], imp[3], cr[3], dw[3];
    for (int k = 0; k < 3; ++k) diff[k] = pb[k] - pa[k];                   /* :100 */
    const REAL dist = FN(np_norm3)(diff);                                   /* :101 */
    for (int k = 0; k < 3; ++k) nrm[k] = diff[k] / (dist + (REAL)1e-8);    /* :104 */
    for (int k = 0; k < 3; ++k) cp[k] = (pa[k] + pb[k]) / (REAL)2;         /* :105 */
    for (int k = 0; k < 3; ++k) { r1[k] = cp[k] - pa[k]; r2[k] = cp[k] - pb[k]; }   /* :106-107 */
    FN(rbo_pair_impulse)(ma, Ia, va, wa, r1, nrm, e, mu, imp);              /* :109-110 */
    const REAL corr = (((ra + rb) + tol) - dist) / (REAL)2;                 /* :116 */
    if (self_is_a) {
        FN(np_cross)(r1, imp, cr);
        FN(np_matvec3)(Ia, cr, dw);
        for (int k = 0; k < 3; ++k) {
            v[k] = v[k] + imp[k] / ma;                                      /* :111 */
            w[k] = w[k] + dw[k];                                            /* :112 */
            p[k] = p[k] - corr * nrm[k];                                    /* :117 */
        }
    } else {
        FN(np_cross)(r2, imp, cr);
        FN(np_matvec3)(Ib, cr, dw);
        for (int k = 0; k < 3; ++k) {
            v[k] = v[k] - imp[k] / mb;                                      /* :113 */
            w[k] = w[k] - dw[k];                                            /* :114 */
            p[k] = p[k] + corr * nrm[k];                                    /* :118 */
        }
    }
}

/* ball-ball test of ball_collision.py:100-103 for the pair (a < b) */
static inline int FN(ball_pair_hit)(const REAL pa[3], REAL ra, const REAL pb[3], REAL rb, REAL tol) {
    REAL diff[3];
    for (int k = 0; k < 3; ++k) diff[k] = pb[k] - pa[k];
    return FN(np_norm3)(diff) < (ra + rb) + tol;
}

/* nsteps of the ball law on AoS qpos[N*7] / qvel[N*6] (in place); spheres
 * only; ground = the z = 0 plane (n_planes >= 1).  Optionally the pair
 * lists of the last step (CSR over all balls, partners ascending). */
int FN(rbo_pair_step)(const rb_scene_desc *d, double *qpos, double *qvel, int64_t nsteps, double dt_,
                      double e_, double mu_, double tol_, int32_t *out_counts, int32_t *out_partner,
                      int64_t out_cap, int64_t *out_total) {
    const int64_t N = d->n_bodies;
    const int maxp = d->max_partners > 0 ? d->max_partners : 16;
    const REAL dt = (REAL)dt_, e = (REAL)e_, mu = (REAL)mu_, tol = (REAL)tol_;
    const REAL g[3] = {(REAL)d->gravity[0], (REAL)d->gravity[1], (REAL)d->gravity[2]};
    const int ground = d->n_planes > 0;
    for (int64_t i = 0; i < N; ++i)
        if (d->kind[i] != RB_BODY_SPHERE) return RB_EUNSUPPORTED;
    REAL *p = (REAL *)malloc(sizeof(REAL) * 3 * (size_t)(N + 1));       /* post-ground */
    REAL *vw = (REAL *)malloc(sizeof(REAL) * 6 * (size_t)(N + 1));
    REAL *np_ = (REAL *)malloc(sizeof(REAL) * 3 * (size_t)(N + 1));     /* end of step */
    REAL *nvw = (REAL *)malloc(sizeof(REAL) * 6 * (size_t)(N + 1));
    REAL *Iinv = (REAL *)malloc(sizeof(REAL) * 9 * (size_t)(N + 1));
    REAL *rad = (REAL *)malloc(sizeof(REAL) * (size_t)(N + 1));
    int32_t *cnt = (int32_t *)calloc((size_t)(N + 1), sizeof(int32_t));
    int32_t *lst = (int32_t *)malloc(sizeof(int32_t) * (size_t)maxp * (size_t)(N + 1));
    FN(cellrec) *cells = (FN(cellrec) *)malloc(sizeof(FN(cellrec)) * (size_t)(N + 1));
    int64_t *ix = (int64_t *)malloc(sizeof(int64_t) * 3 * (size_t)(N + 1));
    int rc = RB_OK;
    if (!p || !vw || !np_ || !nvw || !Iinv || !rad || !cnt || !lst || !cells || !ix) { rc = RB_ENOMEM; goto out; }
    REAL rmax = 0;
    for (int64_t i = 0; i < N; ++i) {
        rad[i] = (REAL)d->size[3 * i];
        if (rad[i] > rmax) rmax = rad[i];
        FN(rbo_ball_iinv)((REAL)d->mass[i], rad[i], Iinv + 9 * i);
        for (int k = 0; k < 3; ++k) np_[3 * i + k] = (REAL)qpos[7 * i + k];
        for (int k = 0; k < 6; ++k) nvw[6 * i + k] = (REAL)qvel[6 * i + k];
    }
    const REAL cs = ((REAL)2 * rmax + tol) * (REAL)1.001;
    for (int64_t step = 0; step < nsteps; ++step) {
        /* ground phase of every ball from its own state */
        for (int64_t i = 0; i < N; ++i) {
            for (int k = 0; k < 3; ++k) p[3 * i + k] = np_[3 * i + k];
            for (int k = 0; k < 6; ++k) vw[6 * i + k] = nvw[6 * i + k];
            FN(ball_ground)(p + 3 * i, vw + 6 * i, vw + 6 * i + 3, (REAL)d->mass[i], rad[i], Iinv + 9 * i, g,
                            dt, e, mu, ground);
        }
        /* pairs on post-ground positions: exact cells of size >= reach */
        for (int64_t i = 0; i < N; ++i) {
            for (int k = 0; k < 3; ++k) {
                const REAL c = p[3 * i + k];
                if (!(c == c) || FABS(c) > cs * (REAL)1000000) { rc = RB_EDOM; goto out; }
                ix[3 * i + k] = (int64_t)floor((double)(c / cs));
            }
            cells[i].key = FN(cell_key)(ix[3 * i], ix[3 * i + 1], ix[3 * i + 2]);
            cells[i].id = i;
        }
        qsort(cells, (size_t)N, sizeof(FN(cellrec)), FN(cell_cmp));
        for (int64_t i = 0; i < N; ++i) {
            int n = 0;
            for (int dx = -1; dx <= 1; ++dx)
                for (int dy = -1; dy <= 1; ++dy)
                    for (int dz = -1; dz <= 1; ++dz) {
                        FN(cellrec) probe = {FN(cell_key)(ix[3 * i] + dx, ix[3 * i + 1] + dy, ix[3 * i + 2] + dz), -1};
                        int64_t lo = 0, hi = N;
                        while (lo < hi) {
                            int64_t mid = (lo + hi) / 2;
                            if (FN(cell_cmp)(&cells[mid], &probe) < 0) lo = mid + 1; else hi = mid;
                        }
                        for (int64_t t = lo; t < N && cells[t].key == probe.key; ++t) {
                            const int64_t j = cells[t].id;
                            if (j == i) continue;
                            const int64_t a = i < j ? i : j, b = i < j ? j : i;
                            if (!FN(ball_pair_hit)(p + 3 * a, rad[a], p + 3 * b, rad[b], tol)) continue;
                            if (n >= maxp) { rc = RB_EOVERFLOW; goto out; }
                            int s = n++;
                            while (s > 0 && lst[(int64_t)maxp * i + s - 1] > j) {
                                lst[(int64_t)maxp * i + s] = lst[(int64_t)maxp * i + s - 1];
                                --s;
                            }
                            lst[(int64_t)maxp * i + s] = (int32_t)j;
                        }
                    }
            cnt[i] = n;
        }
        /* each ball: its pairs in ascending partner id, then x += v dt */
        for (int64_t i = 0; i < N; ++i) {
            REAL pi[3], vi[3], wi[3];
            for (int k = 0; k < 3; ++k) { pi[k] = p[3 * i + k]; vi[k] = vw[6 * i + k]; wi[k] = vw[6 * i + 3 + k]; }
            for (int s = 0; s < cnt[i]; ++s) {
                const int64_t j = lst[(int64_t)maxp * i + s];
                const int64_t a = i < j ? i : j, b = i < j ? j : i;
                FN(ball_pair_apply)(i == a, p + 3 * a, vw + 6 * a, vw + 6 * a + 3, (REAL)d->mass[a], Iinv + 9 * a,
                                    rad[a], p + 3 * b, (REAL)d->mass[b], Iinv + 9 * b, rad[b], tol, e, mu, pi, vi, wi);
            }
            for (int k = 0; k < 3; ++k) {
                np_[3 * i + k] = pi[k] + vi[k] * dt;                        /* :121-122 */
                nvw[6 * i + k] = vi[k];
                nvw[6 * i + 3 + k] = wi[k];
            }
        }
    }
    for (int64_t i = 0; i < N; ++i) {
        for (int k = 0; k < 3; ++k) qpos[7 * i + k] = (double)np_[3 * i + k];
        for (int k = 0; k < 6; ++k) qvel[6 * i + k] = (double)nvw[6 * i + k];
    }
    if (out_counts && nsteps > 0) {
        int64_t t = 0;
        for (int64_t i = 0; i < N; ++i) {
            out_counts[i] = cnt[i];
            for (int s = 0; s < cnt[i]; ++s, ++t)
                if (t < out_cap) out_partner[t] = lst[(int64_t)maxp * i + s];
        }
        if (out_total) *out_total = t;
        if (t > out_cap) rc = RB_EOVERFLOW;
    }
out:
    free(p); free(vw); free(np_); free(nvw); free(Iinv); free(rad); free(cnt); free(lst); free(cells); free(ix);
    return rc;
}

#undef FN
#undef CAT
#undef CAT_
