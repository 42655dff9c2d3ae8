/*
 * rb_oracle.c — CPU oracle for the rigid-body hot path.
 *
 * TEST INFRASTRUCTURE ONLY — the parity checker.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * liboracle.so, and only to check or time the CPU restatement; the product
 * library librbhip.so does not depend on it.
 *
 * What it restates (reference paths relative to the reference repo root):
 *   rbo_impulse        compute_collision_impulse_friction  src/physics/collision.py:7-48
 *   rbo_apply          apply_impulse_friction              src/physics/physics_utils.py:25-49
 *   rbo_inertia_world  compute_inertia_tensor_world        src/physics/collision.py:51-53
 *   rbo_step           custom_step_with_impulse_collision_friction collision.py:56-102,
 *                      timestep_integration time_integeration.py:13-72, and the N-body
 *                      driver custom_step_multi_sphere multi_sphere_bounce.py:42-92
 *                      (SURVEY D1/D2 fixed: body k -> qpos[7k], contacts by body index)
 *   rbo_pair_step      the two-ball law of src/simulation/ball_collision.py:39-125
 *                      (compute_collision_impulse, step_with_custom_collisions),
 *                      generalised to N balls (rb_oracle_pairs.h)
 *   gen_contacts       MuJoCo mj_forward's collision pipeline for plane-sphere,
 *                      plane-box and sphere-sphere (third-party C, not vendored,
 *                      unpinned; restated from MuJoCo's published primitives).
 * Parity pinning: tests/golden/ holds vectors produced by running the
 * reference's own Python functions (make_golden.py); tests/test_oracle_golden.py
 * checks this oracle against them.  Contact generation and mju_mulQuat have
 * no reference-side pin except the plotted single-sphere trajectory
 * (SURVEY §4), which the golden trajectory reproduces.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rbhip.h"

#define REAL double
#define SFX f64
#define FMA fma
#define SQRT sqrt
#define FABS fabs
#include "rb_oracle_impl.h"
#include "rb_oracle_pairs.h"
#undef REAL
#undef SFX
#undef FMA
#undef SQRT
#undef FABS

#define REAL float
#define SFX f32
#define FMA fmaf
#define SQRT sqrtf
#define FABS fabsf
#include "rb_oracle_impl.h"
#include "rb_oracle_pairs.h"
#undef REAL
#undef SFX
#undef FMA
#undef SQRT
#undef FABS

const char *rbo_version(void) { return "rb_oracle 2 (test infrastructure)"; }

/* OpenMP threads for the per-body loops (the CPU baseline's core count). */
void rbo_set_threads(int n) { omp_set_num_threads(n > 0 ? n : 1); }
int rbo_get_threads(void) { return omp_get_max_threads(); }
