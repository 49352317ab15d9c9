/*
 * oracle/soccer_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker).
 *
 * A scalar, plain-C restatement of the reference's env.step() hot path, compiled twice:
 *   liborc_f64.so  (-DORC_F64): double precision, the reference's own precision
 *                   (Chipmunk cpFloat = double, numpy float64 glue). Pinned against the
 *                   golden vectors captured from the reference glue (tests/golden/).
 *   liborc_f32.so  (-DORC_F32): the fp32 arithmetic contract of the HIP kernel. The GPU
 *                   path must reproduce it bit for bit (tests/test_gpu_parity.py).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library; the product (marl-soccer_amd/) never does.
 *
 * What is restated, and from where:
 *   Game.step orchestration ............ soccer_simulation/game/game.py:378-437
 *   force application .................. game.py:383-397 + Chipmunk cpBodyApplyForceAtLocalPoint
 *   physics step (pymunk Space.step) ... Chipmunk2D 7.0.3 cpSpaceStep / cpArbiter / cpCollision /
 *                                        cpBody (third-party, NOT in /root/reference; pymunk is
 *                                        unpinned in requirements.txt:2 and not installed here)
 *   velocity callbacks ................. game/entities.py:19-28 (agent), :69-77 (ball)
 *   goal detection ..................... game.py:401-412
 *   reward shaping ..................... game.py:251-256, 324-375
 *   soft reset / spawn modes ........... game.py:120-249 (numpy PCG64 draws)
 *   terminal override .................. game.py:424-433
 *   observations ....................... game.py:258-322, cast to fp32 by soccer_env.py:131
 *   frame stacking ..................... soccer_env.py:90-96, 130-140
 *   vec auto-reset ..................... marl_vecenv.py:39-53
 *
 * Deliberate restatement choices (DESIGN.md "Physics restatement"):
 *   - Chipmunk's arbiter order follows its BBTree traversal, which cannot be known
 *     offline; arbiters are solved in the canonical shape-pair order of DESIGN.md.
 *   - GJK/EPA closest points are replaced by the analytic closest features of the
 *     circle/segment/box shapes involved (same normal and signed distance up to rounding).
 *   - Contact feature hashes are exact feature ids instead of CP_HASH_PAIR products.
 * Parity of this physics against real Chipmunk is therefore "unpinned"; the glue is pinned.
 */
#include "../include/marl_soccer.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#if defined(ORC_F32)
typedef float real;
#define REAL_MIN FLT_MIN
#define RSQRT(x) sqrtf(x)
#define ORC_NAME "f32"
#elif defined(ORC_F64)
typedef double real;
#define REAL_MIN DBL_MIN
#define RSQRT(x) sqrt(x)
#define ORC_NAME "f64"
#else
#error "define ORC_F32 or ORC_F64"
#endif

#define ORC_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------------------ */
/* Chipmunk cpVect / cpFloat helpers (chipmunk_types.h, cpVect.h semantics)              */
/* ------------------------------------------------------------------------------------ */
typedef struct { real x, y; } vec;
static inline vec v2(real x, real y) { vec r; r.x = x; r.y = y; return r; }
static inline vec vadd(vec a, vec b) { return v2(a.x + b.x, a.y + b.y); }
static inline vec vsub(vec a, vec b) { return v2(a.x - b.x, a.y - b.y); }
static inline vec vneg(vec a) { return v2(-a.x, -a.y); }
static inline vec vmult(vec a, real s) { return v2(a.x * s, a.y * s); }
static inline real vdot(vec a, vec b) { return a.x * b.x + a.y * b.y; }
static inline real vcross(vec a, vec b) { return a.x * b.y - a.y * b.x; }
static inline vec vperp(vec a) { return v2(-a.y, a.x); }
/* c + a * b in the solver (cpArbiterApplyImpulse / ApplyCachedImpulse velocity updates and
 * relative velocities, the impulse rotation). The f32 build is the HIP kernel's contract, which fuses these into
 * fused multiply-adds (one rounding, ms_device.h vmadd); the f64 build keeps Chipmunk's
 * separate multiply and add (the golden fixtures were captured with it). */
#if defined(ORC_F32)
#define SMADD(a, b, c) fmaf((a), (b), (c))
#else
#define SMADD(a, b, c) ((a) * (b) + (c))
#endif
/* used only by the solver and the warm start: the rotation's outer add is fused too */
static inline vec vrotate(vec a, vec b) { return v2(SMADD(a.x, b.x, -(a.y * b.y)), SMADD(a.x, b.y, a.y * b.x)); }
static inline real vlengthsq(vec a) { return vdot(a, a); }
static inline real fmaxr(real a, real b) { return (a > b) ? a : b; }
static inline real fminr(real a, real b) { return (a < b) ? a : b; }
static inline real fclamp(real f, real lo, real hi) { return fminr(fmaxr(f, lo), hi); }
static inline real fclamp01(real f) { return fmaxr((real)0, fminr(f, (real)1)); }
static inline vec vlerp(vec a, vec b, real t) { return vadd(vmult(a, (real)1 - t), vmult(b, t)); }

/* cpCollision.c ClosestT / LerpT (t in [-1, 1]) */
static inline real closest_t(vec a, vec b) {
  vec delta = vsub(b, a);
  return -fclamp(vdot(delta, vadd(a, b)) / vlengthsq(delta), (real)-1, (real)1);
}
static inline vec lerp_t(vec a, vec b, real t) {
  real ht = (real)0.5 * t;
  return vadd(vmult(a, (real)0.5 - ht), vmult(b, (real)0.5 + ht));
}

/* ------------------------------------------------------------------------------------ */
/* fp32 trigonometry contract (the HIP kernel implements the same operations)          */
/* ------------------------------------------------------------------------------------ */
#if defined(ORC_F32)
/* Cody-Waite reduction by pi/2 (3-part split, parts of <= 12 significant bits) and the
 * cephes sinf/cosf minimax polynomials on [-pi/4, pi/4]. No FMA (-ffp-contract=off). */
static void orc_sincos(float x, float *s_out, float *c_out) {
  if (!(x == x) || fabsf(x) > 1.0e30f) { *s_out = NAN; *c_out = NAN; return; }
  float kf = rintf(x * 0.636619746685028076171875f);
  if (kf > 1073741824.0f) kf = 1073741824.0f;
  if (kf < -1073741824.0f) kf = -1073741824.0f;
  int q = (int)kf;
  float r = ((x - kf * 1.5703125f) - kf * 4.838705062866211e-4f) - kf * -4.371138828673793e-8f;
  float z = r * r;
  float sr = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * r + r;
  float cr = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z
             - 0.5f * z + 1.0f;
  switch (q & 3) {
    case 0: *s_out = sr; *c_out = cr; break;
    case 1: *s_out = cr; *c_out = -sr; break;
    case 2: *s_out = -sr; *c_out = -cr; break;
    default: *s_out = -cr; *c_out = sr; break;
  }
}
/* atan2(sin a, cos a) / pi restated as a Cody-Waite wrap of a into [-pi, pi]. */
static float orc_angle_obs(float a) {
  float k = rintf(a * 0.15915493667125702f);
  float w = (a - k * 6.28125f) - k * 0.0019353071693331003f;
  return w / 3.1415927410125732f;
}
#else
/* libm sin and cos called separately, as Chipmunk's cpvforangle and Python's math module
 * do: gcc would otherwise fuse them into glibc sincos(), which differs in the last ulp for
 * ~0.1% of arguments. */
static double (*volatile libm_sin)(double) = sin;
static double (*volatile libm_cos)(double) = cos;
static void orc_sincos(double x, double *s_out, double *c_out) { *s_out = libm_sin(x); *c_out = libm_cos(x); }
static double orc_angle_obs(double a) { return atan2(libm_sin(a), libm_cos(a)) / M_PI; }
#endif

/* ------------------------------------------------------------------------------------ */
/* Parameters                                                                            */
/* ------------------------------------------------------------------------------------ */
enum { B_STATIC = 5 };

typedef struct { vec a, b, n; real r; real bb[4]; } orc_seg;

typedef struct orc_params {
  real dt, slop, bias_coef;
  real m_inv[6], i_inv[6];
  real agent_damp, ball_damp, vmax;
  real force_max, torque_max;
  real obs_vmax, obs_wmax;
  real e_aa, u_aa, e_ab, u_ab, e_aw, u_aw, e_ag, u_ag, e_bw, u_bw;
  real prox_mult, goal_mult, alive, goal_reward, concede_penalty, score_diff_mult;
  int max_steps, autoreset;
  orc_seg seg[8];
} orc_params;

/* segment geometry: game.py:46-72 (walls r=2 e=.95 u=.2; goal lines r=1 e=.95 u=0) */
static const double SEG_DEF[8][5] = {
    {10, 10, 790, 10, 2},   {10, 590, 790, 590, 2}, {10, 10, 10, 225, 2},   {10, 375, 10, 590, 2},
    {790, 10, 790, 225, 2}, {790, 375, 790, 590, 2}, {10, 225, 10, 375, 1}, {790, 225, 790, 375, 1}};

ORC_API void orc_params_init(const ms_config *cfg, orc_params *P) {
  memset(P, 0, sizeof(*P));
#if defined(ORC_F32)
  P->dt = (float)(1.0 / 60.0);
  P->bias_coef = (float)(1.0 - pow(pow(1.0 - 0.1, 60.0), 1.0 / 60.0));
#else
  P->dt = 1.0 / 60.0;
  P->bias_coef = 1.0 - pow(pow(1.0 - 0.1, 60.0), P->dt);
#endif
  P->slop = (real)0.1;
  real am = (real)cfg->agent_mass, bm = (real)cfg->ball_mass;
  real ai = (real)cfg->agent_moment, bi = (real)cfg->ball_moment;
  for (int i = 0; i < 4; ++i) { P->m_inv[i] = (real)1 / am; P->i_inv[i] = (real)1 / ai; }
  P->m_inv[4] = (real)1 / bm; P->i_inv[4] = (real)1 / bi;
  P->m_inv[5] = 0; P->i_inv[5] = 0;
  P->agent_damp = (real)cfg->agent_friction;
  P->ball_damp = (real)cfg->ball_friction;
  P->vmax = (real)cfg->max_velocity;
  P->force_max = (real)cfg->action_force_max;
  P->torque_max = (real)cfg->action_torque_max;
  P->obs_vmax = (real)(cfg->max_velocity > 1e-6 ? cfg->max_velocity : 1e-6);
  P->obs_wmax = (real)(cfg->max_angular_velocity > 1e-6 ? cfg->max_angular_velocity : 1e-6);
  real ea = (real)cfg->agent_elasticity, ua = (real)cfg->agent_surface_friction;
  real eb = (real)cfg->ball_elasticity, ub = (real)cfg->ball_surface_friction;
  real ew = (real)0.95, uw = (real)0.2, eg = (real)0.95, ug = (real)0.0;
  P->e_aa = ea * ea; P->u_aa = ua * ua;
  P->e_ab = eb * ea; P->u_ab = ub * ua;
  P->e_aw = ew * ea; P->u_aw = uw * ua;
  P->e_ag = eg * ea; P->u_ag = ug * ua;
  P->e_bw = eb * ew; P->u_bw = ub * uw;
  P->prox_mult = (real)cfg->ball_proximity_multiplier;
  P->goal_mult = (real)cfg->move_ball_to_goal_multiplier;
  P->alive = (real)cfg->alive_penalty;
  P->goal_reward = (real)cfg->goal_scored_reward;
  P->concede_penalty = (real)cfg->goal_conceded_penalty;
  P->score_diff_mult = (real)cfg->score_difference_multiplier;
  P->max_steps = cfg->max_steps;
  P->autoreset = cfg->autoreset;
  for (int s = 0; s < 8; ++s) {
    orc_seg *g = &P->seg[s];
    g->a = v2((real)SEG_DEF[s][0], (real)SEG_DEF[s][1]);
    g->b = v2((real)SEG_DEF[s][2], (real)SEG_DEF[s][3]);
    g->r = (real)SEG_DEF[s][4];
    vec d = vsub(g->b, g->a); /* cpSegmentShapeInit: n = perp(normalize(b - a)) */
    real len = RSQRT(vdot(d, d));
    g->n = vperp(vmult(d, (real)1 / (len + REAL_MIN)));
    real l, r, bt, t;
    if (g->a.x < g->b.x) { l = g->a.x; r = g->b.x; } else { l = g->b.x; r = g->a.x; }
    if (g->a.y < g->b.y) { bt = g->a.y; t = g->b.y; } else { bt = g->b.y; t = g->a.y; }
    g->bb[0] = l - g->r; g->bb[1] = bt - g->r; g->bb[2] = r + g->r; g->bb[3] = t + g->r;
  }
}

ORC_API void orc_config_default(ms_config *c) {
  memset(c, 0, sizeof(*c));
  c->max_velocity = 200; c->agent_mass = 10; c->ball_mass = 1; c->agent_moment = 100;
  c->ball_moment = 10; c->agent_friction = 0.99; c->ball_friction = 0.97;
  c->agent_elasticity = 0.2; c->agent_surface_friction = 0.8; c->ball_elasticity = 0.95;
  c->ball_surface_friction = 0.2; c->action_force_max = 150000.0; c->action_torque_max = 1000.0;
  c->max_angular_velocity = 1000.0 / 100.0;
  c->ball_proximity_multiplier = 0.002; c->move_ball_to_goal_multiplier = 0.1;
  c->alive_penalty = 0.00001; c->goal_scored_reward = 4.0; c->goal_conceded_penalty = 0.0;
  c->score_difference_multiplier = 0.0; c->max_steps = 1000; c->autoreset = 1;
}

ORC_API int orc_sizeof_params(void) { return (int)sizeof(orc_params); }

/* ------------------------------------------------------------------------------------ */
/* Space: bodies, arbiter cache, per-step arbiter list                                   */
/* ------------------------------------------------------------------------------------ */
typedef struct orc_body {
  real px, py, vx, vy, a, w, vbx, vby, wb, fx, fy, t;
} orc_body;

typedef struct orc_cached {
  int pair, count, idle;
  int hash[2];
  real jn[2], jt[2];
} orc_cached;

typedef struct orc_contact {
  vec r1, r2;
  real nMass, tMass, bias, bounce, jnAcc, jtAcc, jBias;
  real dist; /* ORC_F32: (p2 - p1) . n from the narrowphase frame (see orc_space_phase1) */
  int hash;
} orc_contact;

typedef struct orc_arbiter {
  int pair, ba, bb, count, warm, cache_idx;
  vec n;
  real e, u;
  orc_contact c[2];
} orc_arbiter;

typedef struct orc_space {
  orc_body body[5];
  int n_cache;
  orc_cached cache[MS_MAX_ARBITERS];
  int n_arb;
  orc_arbiter arb[MS_MAX_ARBITERS];
  unsigned long long overflow;
} orc_space;

ORC_API int orc_sizeof_space(void) { return (int)sizeof(orc_space); }
ORC_API int orc_sizeof_body(void) { return (int)sizeof(orc_body); }

/* Shape-pair table (DESIGN.md "pair table"): ids 0-5 agent-agent (i<j), 6-9 ball-agent,
 * 10-41 static-agent (agent-major, 8 statics each), 42-47 ball-wall. For each pair:
 * body a, body b (collision order circle < segment < poly), static index or -1. */
typedef struct { int kind, ba, bb, seg; } pair_def;
enum { K_AA = 0, K_BA = 1, K_SA = 2, K_BS = 3 };
static pair_def pair_table(int p) {
  pair_def d;
  if (p < 6) {
    static const int I[6] = {0, 0, 0, 1, 1, 2}, J[6] = {1, 2, 3, 2, 3, 3};
    d.kind = K_AA; d.ba = I[p]; d.bb = J[p]; d.seg = -1;
  } else if (p < 10) {
    d.kind = K_BA; d.ba = 4; d.bb = p - 6; d.seg = -1;
  } else if (p < 42) {
    d.kind = K_SA; d.ba = B_STATIC; d.bb = (p - 10) / 8; d.seg = (p - 10) % 8;
  } else {
    d.kind = K_BS; d.ba = 4; d.bb = B_STATIC; d.seg = p - 42;
  }
  return d;
}

/* World-space box of an agent (cpPolyShapeCacheData of cpBoxShapeNew(body, 30, 30, 0)):
 * plane i: v[i] = vertex i, n[i] = outward normal of edge v[i-1] -> v[i]. */
typedef struct { vec v[4], n[4]; real bb[4]; } orc_box;

static void box_at(real px, real py, real c, real s, orc_box *o) {
  static const real LX[4] = {15, 15, -15, -15}, LY[4] = {-15, 15, 15, -15};
  for (int i = 0; i < 4; ++i) {
    o->v[i] = v2((c * LX[i] + (-s) * LY[i]) + px, (s * LX[i] + c * LY[i]) + py);
  }
  o->n[0] = v2(s, -c); o->n[1] = v2(c, s); o->n[2] = v2(-s, c); o->n[3] = v2(-c, -s);
  real l = o->v[0].x, r = o->v[0].x, bt = o->v[0].y, t = o->v[0].y;
  for (int i = 1; i < 4; ++i) {
    l = fminr(l, o->v[i].x); r = fmaxr(r, o->v[i].x);
    bt = fminr(bt, o->v[i].y); t = fmaxr(t, o->v[i].y);
  }
  o->bb[0] = l; o->bb[1] = bt; o->bb[2] = r; o->bb[3] = t;
}

static void box_world(const orc_body *b, real c, real s, orc_box *o) { box_at(b->px, b->py, c, s, o); }

static inline int bb_intersects(const real *a, const real *b) {
  return a[0] <= b[2] && b[0] <= a[2] && a[1] <= b[3] && b[1] <= a[3];
}

/* ---- narrowphase output ---- */
typedef struct { vec p1, p2; int hash; } orc_cp;
typedef struct { int count; vec n; orc_cp c[2]; } orc_col;

static void push_contact(orc_col *col, vec p1, vec p2, int hash) {
  col->c[col->count].p1 = p1; col->c[col->count].p2 = p2; col->c[col->count].hash = hash;
  col->count++;
}

/* Edge = two support points with feature ids, a radius (cpCollision.c struct Edge) */
typedef struct { vec a, b; int ha, hb; real r; } orc_edge;

/* SupportEdgeForPoly (cpCollision.c) */
static orc_edge support_edge_box(const orc_box *bx, vec n) {
  int i1 = 0; real mx = -INFINITY;
  for (int i = 0; i < 4; ++i) {
    real d = vdot(bx->v[i], n);
    if (d > mx) { mx = d; i1 = i; }
  }
  int i0 = (i1 + 3) & 3, i2 = (i1 + 1) & 3;
  orc_edge e; e.r = 0;
  if (vdot(n, bx->n[i1]) > vdot(n, bx->n[i2])) {
    e.a = bx->v[i0]; e.ha = i0; e.b = bx->v[i1]; e.hb = i1;
  } else {
    e.a = bx->v[i1]; e.ha = i1; e.b = bx->v[i2]; e.hb = i2;
  }
  return e;
}

/* SupportEdgeForSegment (cpCollision.c) */
static orc_edge support_edge_seg(const orc_seg *s, vec n) {
  orc_edge e; e.r = s->r;
  if (vdot(s->n, n) > 0) { e.a = s->a; e.ha = 0; e.b = s->b; e.hb = 1; }
  else { e.a = s->b; e.ha = 1; e.b = s->a; e.hb = 0; }
  return e;
}

#define FEATURE_HASH(h1, h2) (0x10 | ((h1) << 2) | (h2))

/* ContactPoints (cpCollision.c) */
static void contact_points(orc_edge e1, orc_edge e2, real d, vec n, orc_col *col) {
  real mindist = e1.r + e2.r;
  if (!(d <= mindist)) return;
  col->n = n;
  real d_e1_a = vcross(e1.a, n), d_e1_b = vcross(e1.b, n);
  real d_e2_a = vcross(e2.a, n), d_e2_b = vcross(e2.b, n);
  real e1_denom = (real)1 / (d_e1_b - d_e1_a + REAL_MIN);
  real e2_denom = (real)1 / (d_e2_b - d_e2_a + REAL_MIN);
  {
    vec p1 = vadd(vmult(n, e1.r), vlerp(e1.a, e1.b, fclamp01((d_e2_b - d_e1_a) * e1_denom)));
    vec p2 = vadd(vmult(n, -e2.r), vlerp(e2.a, e2.b, fclamp01((d_e1_a - d_e2_a) * e2_denom)));
    real dist = vdot(vsub(p2, p1), n);
    if (dist <= 0) push_contact(col, p1, p2, FEATURE_HASH(e1.ha, e2.hb));
  }
  {
    vec p1 = vadd(vmult(n, e1.r), vlerp(e1.a, e1.b, fclamp01((d_e2_a - d_e1_a) * e1_denom)));
    vec p2 = vadd(vmult(n, -e2.r), vlerp(e2.a, e2.b, fclamp01((d_e1_b - d_e2_a) * e2_denom)));
    real dist = vdot(vsub(p2, p1), n);
    if (dist <= 0) push_contact(col, p1, p2, FEATURE_HASH(e1.hb, e2.ha));
  }
}

/* CircleToSegment (cpCollision.c), circle = ball (a), segment (b) */
static void col_circle_seg(vec center, real cr, const orc_seg *s, orc_col *col) {
  vec seg_delta = vsub(s->b, s->a);
  real closest_tt = fclamp01(vdot(seg_delta, vsub(center, s->a)) / vlengthsq(seg_delta));
  vec closest = vadd(s->a, vmult(seg_delta, closest_tt));
  real mindist = cr + s->r;
  vec delta = vsub(closest, center);
#if defined(ORC_F32)
  /* an interior closest point is the centre's foot on the segment's line: closest - centre =
   * n_s (n_s . (a - centre)), the same vector without the ~ulp(|b - a|) tangential residue that
   * a + (b - a) t - centre keeps in fp32 (6e-5 px on a 780-px wall tilts the normal by 6e-6) */
  if (closest_tt > (real)0 && closest_tt < (real)1) {
    delta = vmult(s->n, vdot(s->n, vsub(s->a, center)));
    closest = vadd(center, delta);
  }
#endif
  real distsq = vlengthsq(delta);
  if (distsq < mindist * mindist) {
    real dist = RSQRT(distsq);
    vec n = (dist != 0) ? vmult(delta, (real)1 / dist) : s->n;
    col->n = n;
    push_contact(col, vadd(center, vmult(n, cr)), vadd(closest, vmult(n, -s->r)), 0);
  }
}

/* Closest point of point c to the box boundary; returns squared distance, writes the
 * closest box point, the edge index and the ClosestT parameter. Edge i = v[i-1] -> v[i]. */
static real point_box_closest(vec c, const orc_box *bx, vec *pb, int *edge, real *tt) {
  real best = INFINITY;
  for (int i = 0; i < 4; ++i) {
    vec v0 = bx->v[(i + 3) & 3], v1 = bx->v[i];
    vec a = vsub(v0, c), b = vsub(v1, c);
    real t = closest_t(a, b);
    vec p = lerp_t(a, b, t);
    real d2 = vlengthsq(p);
    if (d2 < best) { best = d2; *pb = lerp_t(v0, v1, t); *edge = i; *tt = t; }
  }
  return best;
}

/* CircleToPoly restated: signed distance + normal from the circle centre to the box. */
static void col_circle_box(vec c, real cr, const orc_box *bx, orc_col *col) {
  int fi = 0; real smax = -INFINITY;
  for (int i = 0; i < 4; ++i) {
    real s = vdot(bx->n[i], c) - vdot(bx->n[i], bx->v[i]);
    if (s > smax) { smax = s; fi = i; }
  }
  if (!(smax <= cr)) return;
  vec n, pb; real d;
  if (smax <= 0) { /* centre inside the box: EPA -> least-penetration face */
    vec v0 = bx->v[(fi + 3) & 3], v1 = bx->v[fi];
    real t = closest_t(vsub(v0, c), vsub(v1, c));
    pb = lerp_t(v0, v1, t);
    n = vneg(bx->n[fi]);
    d = smax;
  } else { /* separated: GJK closest features */
    int ei = 0; real t = 0;
    point_box_closest(c, bx, &pb, &ei, &t);
    vec p = vsub(pb, c);
    if (t > (real)-1 && t < (real)1) {
      n = vneg(bx->n[ei]);
      d = vdot(n, p);
    } else {
      d = RSQRT(vlengthsq(p));
      n = vmult(p, (real)1 / (d + REAL_MIN));
    }
  }
  if (d <= cr) {
    col->n = n;
    push_contact(col, vadd(c, vmult(n, cr)), pb, 0);
  }
}

/* SegmentToPoly restated: (n, d) from SAT (overlap) or closest features (separated),
 * then SupportEdgeForSegment / SupportEdgeForPoly / ContactPoints as Chipmunk. */
static void col_seg_box(const orc_seg *s, const orc_box *bx, orc_col *col) {
  real smax = -INFINITY; vec axis = v2(0, 0);
  /* segment faces +n, -n */
  for (int k = 0; k < 2; ++k) {
    vec sn = k == 0 ? s->n : vneg(s->n);
    real m = INFINITY;
    for (int j = 0; j < 4; ++j) m = fminr(m, vdot(sn, bx->v[j]));
    real sep = m - vdot(sn, s->a);
    if (sep > smax) { smax = sep; axis = sn; }
  }
  /* box faces: axis points from segment to box = -n_i */
  for (int i = 0; i < 4; ++i) {
    real m = fminr(vdot(bx->n[i], s->a), vdot(bx->n[i], s->b));
    real sep = m - vdot(bx->n[i], bx->v[i]);
    if (sep > smax) { smax = sep; axis = vneg(bx->n[i]); }
  }
  if (!(smax <= s->r)) return;
  vec n; real d;
  if (smax <= 0) {
    n = axis; d = smax;
  } else {
    /* separated by 0 < d <= r: closest features between the segment core and the box */
    real best = INFINITY; vec pa = v2(0, 0), pb = v2(0, 0); int kind = 0; /* 0 vertex-vertex */
    vec fn = v2(0, 0);
    for (int k = 0; k < 2; ++k) { /* segment endpoints vs box edges */
      vec e = k == 0 ? s->a : s->b;
      for (int i = 0; i < 4; ++i) {
        vec v0 = bx->v[(i + 3) & 3], v1 = bx->v[i];
        vec a = vsub(v0, e), b = vsub(v1, e);
        real t = closest_t(a, b);
        vec p = lerp_t(a, b, t);
        real d2 = vlengthsq(p);
        if (d2 < best) {
          best = d2; pa = e; pb = lerp_t(v0, v1, t);
          if (t > (real)-1 && t < (real)1) { kind = 1; fn = vneg(bx->n[i]); } else kind = 0;
        }
      }
    }
    for (int j = 0; j < 4; ++j) { /* box vertices vs the segment */
      vec a = vsub(s->a, bx->v[j]), b = vsub(s->b, bx->v[j]);
      real t = closest_t(a, b);
      vec p = lerp_t(a, b, t);
      real d2 = vlengthsq(p);
      if (d2 < best) {
        best = d2; pa = lerp_t(s->a, s->b, t); pb = bx->v[j];
        if (t > (real)-1 && t < (real)1) {
          kind = 1;
          fn = (vdot(s->n, vsub(bx->v[j], s->a)) > 0) ? s->n : vneg(s->n);
        } else kind = 0;
      }
    }
    vec p = vsub(pb, pa);
    if (kind) { n = fn; d = vdot(n, p); }
    else { d = RSQRT(vlengthsq(p)); n = vmult(p, (real)1 / (d + REAL_MIN)); }
  }
  if (d - s->r - (real)0 <= 0) {
    contact_points(support_edge_seg(s, n), support_edge_box(bx, vneg(n)), d, n, col);
  }
}

/* PolyToPoly restated: SAT over both boxes' face normals. */
static void col_box_box(const orc_box *A, const orc_box *B, orc_col *col) {
  real smax = -INFINITY; vec axis = v2(0, 0);
  for (int i = 0; i < 4; ++i) {
    real m = INFINITY;
    for (int j = 0; j < 4; ++j) m = fminr(m, vdot(A->n[i], B->v[j]));
    real sep = m - vdot(A->n[i], A->v[i]);
    if (sep > smax) { smax = sep; axis = A->n[i]; }
  }
  for (int i = 0; i < 4; ++i) {
    real m = INFINITY;
    for (int j = 0; j < 4; ++j) m = fminr(m, vdot(B->n[i], A->v[j]));
    real sep = m - vdot(B->n[i], B->v[i]);
    if (sep > smax) { smax = sep; axis = vneg(B->n[i]); }
  }
  if (!(smax - (real)0 - (real)0 <= 0)) return;
  contact_points(support_edge_box(A, axis), support_edge_box(B, vneg(axis)), smax, axis, col);
}

/* ------------------------------------------------------------------------------------ */
/* cpSpaceStep restated, split where Chipmunk calls body->velocity_func                 */
/* ------------------------------------------------------------------------------------ */
static inline real k_scalar_body(real m_inv, real i_inv, vec r, vec n) {
  real rcn = vcross(r, n);
  return m_inv + i_inv * rcn * rcn;
}

static inline vec vmadd(vec a, real s, vec c) { return v2(SMADD(a.x, s, c.x), SMADD(a.y, s, c.y)); }

static void apply_impulse(orc_body *b, real m_inv, real i_inv, vec j, vec r) {
  b->vx = SMADD(j.x, m_inv, b->vx);
  b->vy = SMADD(j.y, m_inv, b->vy);
  b->w = SMADD(i_inv, vcross(r, j), b->w);
}
static void apply_bias_impulse(orc_body *b, real m_inv, real i_inv, vec j, vec r) {
  b->vbx = SMADD(j.x, m_inv, b->vbx);
  b->vby = SMADD(j.y, m_inv, b->vby);
  b->wb = SMADD(i_inv, vcross(r, j), b->wb);
}

/* Phase 1: position integration, collision detection, arbiter update, prestep.
 * (cpSpaceStep up to, not including, the velocity integration.) */
ORC_API void orc_space_phase1(orc_space *sp, const orc_params *P) {
  orc_body stat; memset(&stat, 0, sizeof(stat));
  orc_body *B[6];
  for (int i = 0; i < 5; ++i) B[i] = &sp->body[i];
  B[5] = &stat;
  const real dt = P->dt;

  /* cpBodyUpdatePosition */
  for (int i = 0; i < 5; ++i) {
    orc_body *b = B[i];
    b->px = b->px + (b->vx + b->vbx) * dt;
    b->py = b->py + (b->vy + b->vby) * dt;
    if (i < 4) b->a = b->a + (b->w + b->wb) * dt; /* ball angle unobservable: not tracked */
    b->vbx = 0; b->vby = 0; b->wb = 0;
  }

  /* shape caches (cpShapeUpdateFunc) */
  orc_box box[4];
  real bc[4], bs[4]; /* ORC_F32: each pair's boxes are rebuilt in the pair's frame */
  for (int i = 0; i < 4; ++i) {
    real s, c; orc_sincos(B[i]->a, &s, &c);
    bc[i] = c; bs[i] = s;
    box_world(B[i], c, s, &box[i]);
  }
#if !defined(ORC_F32)
  (void)bc; (void)bs;
#endif
  vec ballc = v2(B[4]->px, B[4]->py);
  const real BR = 10;
  real ballbb[4] = {ballc.x - BR, ballc.y - BR, ballc.x + BR, ballc.y + BR};

  /* collide all shape pairs in canonical order (cpSpaceCollideShapes). The AABB test
   * (broadphase) is in world coordinates. ORC_F32 (the kernel's contract): the narrowphase of
   * a pair runs in the frame of one of its bodies, the origin moved to body a's centre (to the
   * agent's when body a is static), so every coordinate it handles is small (tens of px) and the
   * lever arms r1 = p1 - o_a, r2 = p2 - o_b and the separation (p2 - p1) . n carry fp32
   * rounding of ~1e-6 px instead of the ~5e-5 px of world coordinates near x = 800; the
   * static body's lever arm is never used (zero mass, moment and velocity). ORC_F64 (the
   * reference's precision) keeps Chipmunk's world-frame formulation. */
  sp->n_arb = 0;
  for (int p = 0; p < MS_N_PAIRS; ++p) {
    pair_def pd = pair_table(p);
    orc_col col; col.count = 0; col.n = v2(0, 0);
    real e, u;
    vec oa = v2(0, 0), ob = v2(0, 0); /* the bodies' centres in the narrowphase frame (the
                                         * origin body's is exactly 0) */
#if defined(ORC_F32)
    orc_box ra, rb;
    orc_seg rs;
#endif
    switch (pd.kind) {
      case K_AA:
        if (!bb_intersects(box[pd.ba].bb, box[pd.bb].bb)) continue;
#if defined(ORC_F32)
        { /* frame of agent a */
          real ox = B[pd.ba]->px, oy = B[pd.ba]->py;
          box_at(0, 0, bc[pd.ba], bs[pd.ba], &ra);
          ob = v2(B[pd.bb]->px - ox, B[pd.bb]->py - oy);
          box_at(ob.x, ob.y, bc[pd.bb], bs[pd.bb], &rb);
          col_box_box(&ra, &rb, &col);
        }
#else
        col_box_box(&box[pd.ba], &box[pd.bb], &col);
#endif
        e = P->e_aa; u = P->u_aa;
        break;
      case K_BA:
        if (!bb_intersects(ballbb, box[pd.bb].bb)) continue;
#if defined(ORC_F32)
        { /* frame of the ball */
          real ox = ballc.x, oy = ballc.y;
          ob = v2(B[pd.bb]->px - ox, B[pd.bb]->py - oy);
          box_at(ob.x, ob.y, bc[pd.bb], bs[pd.bb], &rb);
          col_circle_box(oa, BR, &rb, &col);
        }
#else
        col_circle_box(ballc, BR, &box[pd.bb], &col);
#endif
        e = P->e_ab; u = P->u_ab;
        break;
      case K_SA:
        if (!bb_intersects(P->seg[pd.seg].bb, box[pd.bb].bb)) continue;
#if defined(ORC_F32)
        { /* frame of the agent (body b; body a is static) */
          real ox = B[pd.bb]->px, oy = B[pd.bb]->py;
          rs = P->seg[pd.seg];
          rs.a = v2(rs.a.x - ox, rs.a.y - oy);
          rs.b = v2(rs.b.x - ox, rs.b.y - oy);
          box_at(0, 0, bc[pd.bb], bs[pd.bb], &rb);
          col_seg_box(&rs, &rb, &col);
        }
#else
        col_seg_box(&P->seg[pd.seg], &box[pd.bb], &col);
#endif
        if (pd.seg < 6) { e = P->e_aw; u = P->u_aw; } else { e = P->e_ag; u = P->u_ag; }
        break;
      default: /* K_BS: ball vs wall (goal lines are filtered out by the ball's mask) */
        if (!bb_intersects(ballbb, P->seg[pd.seg].bb)) continue;
#if defined(ORC_F32)
        { /* frame of the ball (body a; body b is static) */
          real ox = ballc.x, oy = ballc.y;
          rs = P->seg[pd.seg];
          rs.a = v2(rs.a.x - ox, rs.a.y - oy);
          rs.b = v2(rs.b.x - ox, rs.b.y - oy);
          col_circle_seg(oa, BR, &rs, &col);
        }
#else
        col_circle_seg(ballc, BR, &P->seg[pd.seg], &col);
#endif
        e = P->e_bw; u = P->u_bw;
        break;
    }
    if (col.count == 0) continue;
    if (sp->n_arb >= MS_MAX_ARBITERS) { sp->overflow++; continue; }
    /* cpHashSetInsert on the cached arbiters + cpArbiterUpdate */
    int ci = -1;
    for (int k = 0; k < sp->n_cache; ++k)
      if (sp->cache[k].pair == p) { ci = k; break; }
    orc_arbiter *arb = &sp->arb[sp->n_arb++];
    arb->pair = p; arb->ba = pd.ba; arb->bb = pd.bb; arb->count = col.count;
    arb->cache_idx = ci;
    arb->warm = (ci >= 0 && sp->cache[ci].idle == 0); /* touched last step: NORMAL state */
    arb->n = col.n; arb->e = e; arb->u = u;
    for (int k = 0; k < col.count; ++k) {
      orc_contact *con = &arb->c[k];
#if defined(ORC_F32)
      con->r1 = vsub(col.c[k].p1, oa);
      con->r2 = vsub(col.c[k].p2, ob);
      con->dist = vdot(vsub(col.c[k].p2, col.c[k].p1), col.n);
#else
      (void)oa; (void)ob;
      con->r1 = vsub(col.c[k].p1, v2(B[pd.ba]->px, B[pd.ba]->py));
      con->r2 = vsub(col.c[k].p2, v2(B[pd.bb]->px, B[pd.bb]->py));
      con->dist = 0;
#endif
      con->hash = col.c[k].hash;
      con->jnAcc = 0; con->jtAcc = 0;
      if (ci >= 0) {
        const orc_cached *old = &sp->cache[ci];
        for (int j = 0; j < old->count; ++j)
          if (old->hash[j] == con->hash) { con->jnAcc = old->jn[j]; con->jtAcc = old->jt[j]; }
      }
    }
  }

  /* cpArbiterPreStep (velocities are still the previous step's post-solve values) */
  for (int k = 0; k < sp->n_arb; ++k) {
    orc_arbiter *arb = &sp->arb[k];
    orc_body *a = B[arb->ba], *b = B[arb->bb];
    real ma = P->m_inv[arb->ba], ia = P->i_inv[arb->ba];
    real mb = P->m_inv[arb->bb], ib = P->i_inv[arb->bb];
    vec n = arb->n;
    vec body_delta = v2(b->px - a->px, b->py - a->py);
    for (int i = 0; i < arb->count; ++i) {
      orc_contact *con = &arb->c[i];
      con->nMass = (real)1 / (k_scalar_body(ma, ia, con->r1, n) + k_scalar_body(mb, ib, con->r2, n));
      vec t = vperp(n);
      con->tMass = (real)1 / (k_scalar_body(ma, ia, con->r1, t) + k_scalar_body(mb, ib, con->r2, t));
#if defined(ORC_F32)
      real dist = con->dist; /* (p2 - p1) . n in the narrowphase frame */
      (void)body_delta;
#else
      real dist = vdot(vadd(vsub(con->r2, con->r1), body_delta), n);
#endif
      con->bias = -P->bias_coef * fminr((real)0, dist + P->slop) / dt;
      con->jBias = 0;
      vec v1 = vadd(v2(a->vx, a->vy), vmult(vperp(con->r1), a->w));
      vec v2s = vadd(v2(b->vx, b->vy), vmult(vperp(con->r2), b->w));
      con->bounce = vdot(vsub(v2s, v1), n) * arb->e;
    }
  }
}

/* Default cpBodyUpdateVelocity (gravity 0, damping 1) followed by the reference's
 * custom velocity_func: entities.py:19-28 (agents) and :69-77 (ball). */
ORC_API void orc_space_update_velocities(orc_space *sp, const orc_params *P) {
  const real dt = P->dt;
  for (int i = 0; i < 5; ++i) {
    orc_body *b = &sp->body[i];
    /* v = v*damping + (gravity + f*m_inv)*dt with space damping 1 and gravity 0 */
    b->vx = b->vx * (real)1 + ((real)0 + b->fx * P->m_inv[i]) * dt;
    b->vy = b->vy * (real)1 + ((real)0 + b->fy * P->m_inv[i]) * dt;
    b->w = b->w * (real)1 + b->t * P->i_inv[i] * dt;
    b->fx = 0; b->fy = 0; b->t = 0;
    real damp = i < 4 ? P->agent_damp : P->ball_damp;
    b->vx = b->vx * damp;
    b->vy = b->vy * damp;
    if (i < 4) b->w = b->w * damp;
    real len = RSQRT(b->vx * b->vx + b->vy * b->vy);
    if (len > P->vmax) {
      b->vx = (b->vx / len) * P->vmax;
      b->vy = (b->vy / len) * P->vmax;
    }
  }
}

/* Phase 2: warm start, 10 solver iterations, arbiter cache bookkeeping. */
ORC_API void orc_space_phase2(orc_space *sp, const orc_params *P) {
  orc_body stat; memset(&stat, 0, sizeof(stat));
  orc_body *B[6];
  for (int i = 0; i < 5; ++i) B[i] = &sp->body[i];
  B[5] = &stat;

  /* cpArbiterApplyCachedImpulse (dt_coef = dt/prev_dt = 1) */
  for (int k = 0; k < sp->n_arb; ++k) {
    orc_arbiter *arb = &sp->arb[k];
    if (!arb->warm) continue;
    orc_body *a = B[arb->ba], *b = B[arb->bb];
    for (int i = 0; i < arb->count; ++i) {
      orc_contact *con = &arb->c[i];
      vec j = vrotate(arb->n, v2(con->jnAcc, con->jtAcc));
      apply_impulse(a, P->m_inv[arb->ba], P->i_inv[arb->ba], vneg(j), con->r1);
      apply_impulse(b, P->m_inv[arb->bb], P->i_inv[arb->bb], j, con->r2);
    }
  }

  /* cpArbiterApplyImpulse x iterations (10, pymunk Space default) */
  for (int it = 0; it < 10; ++it) {
    for (int k = 0; k < sp->n_arb; ++k) {
      orc_arbiter *arb = &sp->arb[k];
      orc_body *a = B[arb->ba], *b = B[arb->bb];
      real ma = P->m_inv[arb->ba], ia = P->i_inv[arb->ba];
      real mb = P->m_inv[arb->bb], ib = P->i_inv[arb->bb];
      vec n = arb->n;
      real friction = arb->u;
      for (int i = 0; i < arb->count; ++i) {
        orc_contact *con = &arb->c[i];
        real nMass = con->nMass;
        vec r1 = con->r1, r2 = con->r2;
        vec vb1 = vmadd(vperp(r1), a->wb, v2(a->vbx, a->vby));
        vec vb2 = vmadd(vperp(r2), b->wb, v2(b->vbx, b->vby));
        vec vs1 = vmadd(vperp(r1), a->w, v2(a->vx, a->vy));
        vec vs2 = vmadd(vperp(r2), b->w, v2(b->vx, b->vy));
        vec vr = vsub(vs2, vs1);
        real vbn = vdot(vsub(vb2, vb1), n);
        real vrn = vdot(vr, n);
        real vrt = vdot(vr, vperp(n));

        real jbn = (con->bias - vbn) * nMass;
        real jbnOld = con->jBias;
        con->jBias = fmaxr(jbnOld + jbn, (real)0);

        real jn = -(con->bounce + vrn) * nMass;
        real jnOld = con->jnAcc;
        con->jnAcc = fmaxr(jnOld + jn, (real)0);

        real jtMax = friction * con->jnAcc;
        real jt = -vrt * con->tMass;
        real jtOld = con->jtAcc;
        con->jtAcc = fclamp(jtOld + jt, -jtMax, jtMax);

        vec jb = vmult(n, con->jBias - jbnOld);
        apply_bias_impulse(a, ma, ia, vneg(jb), r1);
        apply_bias_impulse(b, mb, ib, jb, r2);
        vec j = vrotate(n, v2(con->jnAcc - jnOld, con->jtAcc - jtOld));
        apply_impulse(a, ma, ia, vneg(j), r1);
        apply_impulse(b, mb, ib, j, r2);
      }
    }
  }

  /* cpSpaceArbiterSetFilter: touched arbiters idle = 0, others age; drop at persistence 3.
   * The cache stays sorted by pair id. */
  orc_cached nc[MS_MAX_ARBITERS];
  int nn = 0, ia = 0, ic = 0;
  while (ia < sp->n_arb || ic < sp->n_cache) {
    int pa = ia < sp->n_arb ? sp->arb[ia].pair : 1 << 30;
    int pc = ic < sp->n_cache ? sp->cache[ic].pair : 1 << 30;
    orc_cached ent;
    if (pa <= pc) {
      const orc_arbiter *arb = &sp->arb[ia];
      ent.pair = arb->pair; ent.count = arb->count; ent.idle = 0;
      for (int i = 0; i < 2; ++i) {
        ent.hash[i] = i < arb->count ? arb->c[i].hash : 0;
        ent.jn[i] = i < arb->count ? arb->c[i].jnAcc : 0;
        ent.jt[i] = i < arb->count ? arb->c[i].jtAcc : 0;
      }
      ia++;
      if (pa == pc) ic++;
    } else {
      ent = sp->cache[ic++];
      ent.idle += 1;
      if (ent.idle >= 3) continue;
    }
    if (nn >= MS_MAX_ARBITERS) { sp->overflow++; continue; }
    nc[nn++] = ent;
  }
  memcpy(sp->cache, nc, sizeof(orc_cached) * (size_t)nn);
  sp->n_cache = nn;
}

ORC_API void orc_space_step(orc_space *sp, const orc_params *P) {
  orc_space_phase1(sp, P);
  orc_space_update_velocities(sp, P);
  orc_space_phase2(sp, P);
}

ORC_API void orc_space_clear_arbiters(orc_space *sp) { sp->n_cache = 0; sp->n_arb = 0; }

/* ------------------------------------------------------------------------------------ */
/* numpy PCG64 (XSL-RR 128/64) + Generator.uniform / integers(0, 4)                      */
/* ------------------------------------------------------------------------------------ */
typedef struct orc_rng {
  uint64_t state_hi, state_lo, inc_hi, inc_lo;
  int has_uint32;
  uint32_t uinteger;
} orc_rng;

typedef unsigned __int128 u128;
static uint64_t pcg_next64(orc_rng *g) {
  const u128 MULT = ((u128)0x2360ED051FC65DA4ULL << 64) | 0x4385DF649FCCF645ULL;
  u128 st = ((u128)g->state_hi << 64) | g->state_lo;
  u128 inc = ((u128)g->inc_hi << 64) | g->inc_lo;
  st = st * MULT + inc;
  g->state_hi = (uint64_t)(st >> 64); g->state_lo = (uint64_t)st;
  uint64_t x = g->state_hi ^ g->state_lo;
  unsigned rot = (unsigned)(g->state_hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}
static uint32_t pcg_next32(orc_rng *g) {
  if (g->has_uint32) { g->has_uint32 = 0; return g->uinteger; }
  uint64_t nx = pcg_next64(g);
  g->has_uint32 = 1; g->uinteger = (uint32_t)(nx >> 32);
  return (uint32_t)(nx & 0xffffffffu);
}
static double rng_uniform(orc_rng *g, double lo, double hi) {
  double u = (double)(pcg_next64(g) >> 11) * (1.0 / 9007199254740992.0);
  return lo + (hi - lo) * u;
}
static int rng_int4(orc_rng *g) { /* integers(0, 4): Lemire on 32 bits, rng_excl = 4 */
  uint64_t m = (uint64_t)pcg_next32(g) * 4u;
  return (int)(m >> 32);
}

/* ------------------------------------------------------------------------------------ */
/* Environment (Game + SoccerEnv + vec-env auto-reset)                                   */
/* ------------------------------------------------------------------------------------ */
/* obs history snapshot (include/marl_soccer.h MS_SNAP_SIZE): px[5], py[5], vx[4], vy[4],
 * angle[4], w[4] — the whole input of Game._get_observations */
typedef struct { real v[MS_SNAP_SIZE]; } orc_snap;

typedef struct orc_env {
  orc_space sp;
  orc_rng rng;
  int steps, score_blue, score_red, mode, hist_empty;
  orc_snap hist[2]; /* [0] = t-2, [1] = t-1 */
} orc_env;

ORC_API int orc_sizeof_env(void) { return (int)sizeof(orc_env); }

static void set_pos(orc_body *b, double x, double y) { b->px = (real)x; b->py = (real)y; }

/* _apply_fixed/_random/_full_random_positions (game.py:129-249) */
static void spawn(orc_env *e, int mode) {
  orc_body *A = e->sp.body, *ball = &e->sp.body[4];
  if (mode == MS_SPAWN_FIXED) {
    set_pos(&A[0], 800 * 0.25, 600 * 0.33); set_pos(&A[1], 800 * 0.25, 600 * 0.66);
    set_pos(&A[2], 800 * 0.75, 600 * 0.33); set_pos(&A[3], 800 * 0.75, 600 * 0.66);
    set_pos(ball, 800 / 2.0, 600 / 2.0);
  } else if (mode == MS_SPAWN_RANDOM) {
    const double margin = 30.0, lxmax = 380.0, rxmin = 420.0, rxmax = 770.0, ymin = 30.0, ymax = 570.0;
    double bx1 = rng_uniform(&e->rng, margin, lxmax), by1 = rng_uniform(&e->rng, ymin, ymax);
    double bx2 = rng_uniform(&e->rng, margin, lxmax), by2 = rng_uniform(&e->rng, ymin, ymax);
    double rx1 = rng_uniform(&e->rng, rxmin, rxmax), ry1 = rng_uniform(&e->rng, ymin, ymax);
    double rx2 = rng_uniform(&e->rng, rxmin, rxmax), ry2 = rng_uniform(&e->rng, ymin, ymax);
    double cx = 400.0 + rng_uniform(&e->rng, -40.0, 40.0);
    double cy = 300.0 + rng_uniform(&e->rng, -40.0, 40.0);
    set_pos(&A[0], bx1, by1); set_pos(&A[1], bx2, by2);
    set_pos(&A[2], rx1, ry1); set_pos(&A[3], rx2, ry2);
    set_pos(ball, cx, cy);
  } else {
    const double lo = 30.0, xmax = 770.0, ymax = 570.0;
    double u0 = rng_uniform(&e->rng, 0.0, 1.0);
    double bx1, by1, bx2, by2;
    if (u0 < 0.75) {
      int c1 = rng_int4(&e->rng), c2 = rng_int4(&e->rng);
      int cs[2] = {c1, c2}; double out[2][2];
      for (int k = 0; k < 2; ++k) {
        int left = cs[k] == 0 || cs[k] == 1, top = cs[k] == 0 || cs[k] == 2;
        double cx = left ? 18.0 : 782.0, cy = top ? 582.0 : 18.0;
        double jx = rng_uniform(&e->rng, -5.0, 5.0), jy = rng_uniform(&e->rng, -5.0, 5.0);
        out[k][0] = cx + jx; out[k][1] = cy + jy;
      }
      bx1 = out[0][0]; by1 = out[0][1]; bx2 = out[1][0]; by2 = out[1][1];
    } else {
      bx1 = rng_uniform(&e->rng, lo, xmax); by1 = rng_uniform(&e->rng, lo, ymax);
      bx2 = rng_uniform(&e->rng, lo, xmax); by2 = rng_uniform(&e->rng, lo, ymax);
    }
    double rx1 = rng_uniform(&e->rng, lo, xmax), ry1 = rng_uniform(&e->rng, lo, ymax);
    double rx2 = rng_uniform(&e->rng, lo, xmax), ry2 = rng_uniform(&e->rng, lo, ymax);
    double cx = rng_uniform(&e->rng, lo, xmax), cy = rng_uniform(&e->rng, lo, ymax);
    set_pos(&A[0], bx1, by1); set_pos(&A[1], bx2, by2);
    set_pos(&A[2], rx1, ry1); set_pos(&A[3], rx2, ry2);
    set_pos(ball, cx, cy);
  }
  for (int i = 0; i < 4; ++i) {
    A[i].vx = 0; A[i].vy = 0; A[i].w = 0;
    A[i].a = i < 2 ? (real)0 : (real)M_PI;
  }
  ball->vx = 0; ball->vy = 0;
}

/* Game._get_observations (game.py:258-322) for one env -> fp32 frame [4][22] */
static void vec_to_unit_mag(real dx, real dy, float *o) {
  real mag = RSQRT(dx * dx + dy * dy);
  if (mag > (real)1e-8) { o[0] = (float)(dx / mag); o[1] = (float)(dy / mag); }
  else { o[0] = 0.0f; o[1] = 0.0f; mag = 0; }
  o[2] = (float)(mag / (real)1000.0); /* field diagonal hypot(800, 600) */
}

static void snapshot(const orc_space *sp, orc_snap *s) {
  for (int b = 0; b < 5; ++b) { s->v[b] = sp->body[b].px; s->v[5 + b] = sp->body[b].py; }
  for (int i = 0; i < 4; ++i) {
    s->v[10 + i] = sp->body[i].vx; s->v[14 + i] = sp->body[i].vy;
    s->v[18 + i] = sp->body[i].a; s->v[22 + i] = sp->body[i].w;
  }
}

static void observe_snap(const orc_snap *sn, const orc_params *P, float frame[4][22]) {
  static const int TEAM[4] = {1, 0, 3, 2};
  static const int OPP[4][2] = {{2, 3}, {2, 3}, {0, 1}, {0, 1}};
  const real *px = sn->v, *py = sn->v + 5, *vx = sn->v + 10, *vy = sn->v + 14, *an = sn->v + 18, *w = sn->v + 22;
  for (int i = 0; i < 4; ++i) {
    float *o = frame[i];
    o[0] = (float)vx[i] / (float)P->obs_vmax;
    o[1] = (float)vy[i] / (float)P->obs_vmax;
    o[2] = (float)orc_angle_obs(an[i]);
    o[3] = (float)(w[i] / P->obs_wmax);
    const int others[4] = {TEAM[i], OPP[i][0], OPP[i][1], 4};
    for (int k = 0; k < 4; ++k) vec_to_unit_mag(px[others[k]] - px[i], py[others[k]] - py[i], o + 4 + 3 * k);
    real own_x = i < 2 ? (real)10 : (real)790, opp_x = i < 2 ? (real)790 : (real)10;
    vec_to_unit_mag(own_x - px[i], (real)300 - py[i], o + 16);
    vec_to_unit_mag(opp_x - px[i], (real)300 - py[i], o + 19);
  }
}

ORC_API void orc_observe_space(const orc_space *sp, const orc_params *P, float frame[4][22]) {
  orc_snap s;
  snapshot(sp, &s);
  observe_snap(&s, P, frame);
}

/* prev_d - cur_d for d = |a - b| (game.py:336-338, 344-345), restated as
 * (|p|^2 - |c|^2) / (|p| + |c|) with p - c = db - da computed from displacements. */
static real dist_improvement(real a0x, real a0y, real b0x, real b0y, real a1x, real a1y, real b1x,
                             real b1y) {
  real px = a0x - b0x, py = a0y - b0y;
  real cx = a1x - b1x, cy = a1y - b1y;
  real dax = a1x - a0x, day = a1y - a0y;
  real dbx = b1x - b0x, dby = b1y - b0y;
  real num = (dbx - dax) * (px + cx) + (dby - day) * (py + cy);
  real den = RSQRT(px * px + py * py) + RSQRT(cx * cx + cy * cy);
  return den > 0 ? num / den : (real)0;
}

/* _calculate_rewards + terminal override (game.py:324-375, 424-433). pos: [5][2]. */
static real blue_reward(const orc_params *P, const real prev[5][2], const real cur[5][2], int goal,
                        int terminal, int score_blue, int score_red) {
  if (terminal) return P->score_diff_mult * (real)(score_blue - score_red);
  real r = 0;
  if (P->prox_mult != 0) {
    real imp = dist_improvement(prev[0][0], prev[0][1], prev[4][0], prev[4][1], cur[0][0], cur[0][1],
                                cur[4][0], cur[4][1]) +
               dist_improvement(prev[1][0], prev[1][1], prev[4][0], prev[4][1], cur[1][0], cur[1][1],
                                cur[4][0], cur[4][1]);
    r = r + P->prox_mult * imp;
  }
  real g = dist_improvement(prev[4][0], prev[4][1], 790, 300, cur[4][0], cur[4][1], 790, 300);
  r = r + g * P->goal_mult;
  if (goal == 1) r = r + P->goal_reward;
  else if (goal == 2) r = r - P->concede_penalty;
  r = r - P->alive;
  return r;
}

ORC_API void orc_debug_rewards(const orc_params *P, int n, const float *prev_pos, const float *cur_pos,
                               const int8_t *goal, const uint8_t *terminal, const int32_t *score,
                               double *rew) {
  for (int e = 0; e < n; ++e) {
    real pv[5][2], cu[5][2];
    for (int b = 0; b < 5; ++b)
      for (int k = 0; k < 2; ++k) { pv[b][k] = prev_pos[e * 10 + b * 2 + k]; cu[b][k] = cur_pos[e * 10 + b * 2 + k]; }
    real r = blue_reward(P, pv, cu, goal[e], terminal[e], score[2 * e], score[2 * e + 1]);
    rew[2 * e] = (double)r; rew[2 * e + 1] = (double)r;
  }
}

/* Game.reset (game.py:76-118) + SoccerEnv.reset frame fill (soccer_env.py:90-96). */
ORC_API void orc_env_reset(orc_env *e, const orc_params *P, const uint64_t *pcg, int mode, float *obs) {
  if (pcg) {
    e->rng.state_hi = pcg[0]; e->rng.state_lo = pcg[1];
    e->rng.inc_hi = pcg[2]; e->rng.inc_lo = pcg[3];
    e->rng.has_uint32 = 0; e->rng.uinteger = 0;
  }
  e->mode = mode;
  e->steps = 0; e->score_blue = 0; e->score_red = 0;
  memset(e->sp.body, 0, sizeof(e->sp.body)); /* bodies are re-created: v, w, bias, f, t = 0 */
  orc_space_clear_arbiters(&e->sp);          /* space.remove drops every arbiter */
  spawn(e, mode);
  float f[4][22];
  orc_observe_space(&e->sp, P, f);
  snapshot(&e->sp, &e->hist[0]);
  e->hist[1] = e->hist[0];
  e->hist_empty = 0;
  if (obs)
    for (int i = 0; i < 4; ++i)
      for (int s = 0; s < 3; ++s) memcpy(obs + i * 66 + s * 22, f[i], 22 * sizeof(float));
}

/* One SyncMultiAgentVecEnv/SoccerEnv step for one env. Returns 0, or MS_ERR_NONFINITE_ACTION
 * (state untouched). obs [4][66], rew [4], trunc [4], goal, score [2]. */
ORC_API int orc_env_step(orc_env *e, const orc_params *P, const float *act, float *obs, double *rew,
                         uint8_t *trunc, int8_t *goal_out, int32_t *score_out) {
  for (int k = 0; k < 12; ++k)
    if (!isfinite(act[k])) return MS_ERR_NONFINITE_ACTION;
  /* SoccerEnv.step: clip then scale in fp32 (soccer_env.py:119-125) */
  float F[4][3];
  for (int i = 0; i < 4; ++i) {
    for (int k = 0; k < 3; ++k) {
      float a = act[i * 3 + k];
      a = a < -1.0f ? -1.0f : (a > 1.0f ? 1.0f : a);
      F[i][k] = a * (k < 2 ? (float)P->force_max : (float)P->torque_max);
    }
  }
  orc_body *B = e->sp.body;
  real prev[5][2];
  for (int b = 0; b < 5; ++b) { prev[b][0] = B[b].px; prev[b][1] = B[b].py; }
  e->steps += 1;
  for (int i = 0; i < 4; ++i) {
    real s, c; orc_sincos(B[i].a, &s, &c);
    real fx = (real)F[i][0], fy = (real)F[i][1];
    /* body.force = (0, 0) then cpBodyApplyForceAtWorldPoint: f = 0 + R(angle) F */
    B[i].fx = (real)0 + (c * fx + (-s) * fy);
    B[i].fy = (real)0 + (s * fx + c * fy);
    B[i].t = (real)F[i][2];
  }
  B[4].fx = 0; B[4].fy = 0; B[4].t = 0;
  orc_space_step(&e->sp, P);

  int goal = 0;
  real bx = B[4].px, by = B[4].py;
  if (bx < (real)10 && (real)225 < by && by < (real)375) { goal = 2; e->score_red += 1; }
  else if (bx > (real)790 && (real)225 < by && by < (real)375) { goal = 1; e->score_blue += 1; }
  real cur[5][2];
  for (int b = 0; b < 5; ++b) { cur[b][0] = B[b].px; cur[b][1] = B[b].py; }
  int done = (P->max_steps > 0 && e->steps >= P->max_steps);
  real r = blue_reward(P, prev, cur, goal, 0, 0, 0);
  if (goal) spawn(e, e->mode);
  if (done) r = blue_reward(P, prev, cur, goal, 1, e->score_blue, e->score_red);

  orc_snap now;
  snapshot(&e->sp, &now);
  if (e->hist_empty) { e->hist[0] = now; e->hist[1] = now; e->hist_empty = 0; }
  float f0[4][22], f1[4][22], f[4][22];
  observe_snap(&e->hist[0], P, f0);
  observe_snap(&e->hist[1], P, f1);
  observe_snap(&now, P, f);
  if (obs)
    for (int i = 0; i < 4; ++i) {
      memcpy(obs + i * 66, f0[i], 22 * sizeof(float));
      memcpy(obs + i * 66 + 22, f1[i], 22 * sizeof(float));
      memcpy(obs + i * 66 + 44, f[i], 22 * sizeof(float));
    }
  e->hist[0] = e->hist[1];
  e->hist[1] = now;
  if (rew) { rew[0] = (double)r; rew[1] = (double)r; rew[2] = 0.0; rew[3] = 0.0; }
  if (trunc) for (int i = 0; i < 4; ++i) trunc[i] = (uint8_t)done;
  if (goal_out) *goal_out = (int8_t)goal;
  if (score_out) { score_out[0] = e->score_blue; score_out[1] = e->score_red; }
  if (done && P->autoreset) orc_env_reset(e, P, NULL, MS_SPAWN_FULL_RANDOM, obs);
  return 0;
}

ORC_API void orc_env_observe(const orc_env *e, const orc_params *P, float *frame) {
  orc_observe_space(&e->sp, P, (float(*)[22])frame);
}

/* ---- state record exchange (include/marl_soccer.h ms_env_state) ---- */
ORC_API void orc_env_export(const orc_env *e, ms_env_state *s) {
  memset(s, 0, sizeof(*s));
  for (int b = 0; b < 5; ++b) {
    const orc_body *o = &e->sp.body[b];
    ms_body_state *d = &s->body[b];
    d->px = (float)o->px; d->py = (float)o->py; d->vx = (float)o->vx; d->vy = (float)o->vy;
    d->angle = b < 4 ? (float)o->a : 0.0f; d->w = (float)o->w;
    d->vbx = (float)o->vbx; d->vby = (float)o->vby; d->wb = (float)o->wb;
  }
  for (int k = 0; k < 2; ++k)
    for (int j = 0; j < MS_SNAP_SIZE; ++j) s->snap[k][j] = (float)e->hist[k].v[j];
  s->steps = e->steps; s->score_blue = e->score_blue; s->score_red = e->score_red;
  s->mode = (uint8_t)e->mode; s->hist_empty = (uint8_t)e->hist_empty;
  s->has_uint32 = (uint8_t)e->rng.has_uint32; s->uinteger = e->rng.uinteger;
  s->pcg_state_hi = e->rng.state_hi; s->pcg_state_lo = e->rng.state_lo;
  s->pcg_inc_hi = e->rng.inc_hi; s->pcg_inc_lo = e->rng.inc_lo;
  s->n_arb = (uint8_t)e->sp.n_cache;
  for (int k = 0; k < e->sp.n_cache; ++k) {
    const orc_cached *c = &e->sp.cache[k];
    ms_arbiter_state *a = &s->arb[k];
    a->pair = (uint8_t)c->pair; a->count = (uint8_t)c->count; a->idle = (uint8_t)c->idle;
    for (int i = 0; i < 2; ++i) { a->hash[i] = (uint8_t)c->hash[i]; a->jn[i] = (float)c->jn[i]; a->jt[i] = (float)c->jt[i]; }
  }
}

ORC_API void orc_env_import(orc_env *e, const ms_env_state *s) {
  memset(e, 0, sizeof(*e));
  for (int b = 0; b < 5; ++b) {
    orc_body *o = &e->sp.body[b];
    const ms_body_state *d = &s->body[b];
    o->px = d->px; o->py = d->py; o->vx = d->vx; o->vy = d->vy; o->a = b < 4 ? d->angle : 0;
    o->w = d->w; o->vbx = d->vbx; o->vby = d->vby; o->wb = d->wb;
  }
  for (int k = 0; k < 2; ++k)
    for (int j = 0; j < MS_SNAP_SIZE; ++j) e->hist[k].v[j] = s->snap[k][j];
  e->steps = s->steps; e->score_blue = s->score_blue; e->score_red = s->score_red;
  e->mode = s->mode; e->hist_empty = s->hist_empty;
  e->rng.has_uint32 = s->has_uint32; e->rng.uinteger = s->uinteger;
  e->rng.state_hi = s->pcg_state_hi; e->rng.state_lo = s->pcg_state_lo;
  e->rng.inc_hi = s->pcg_inc_hi; e->rng.inc_lo = s->pcg_inc_lo;
  e->sp.n_cache = s->n_arb;
  for (int k = 0; k < s->n_arb; ++k) {
    orc_cached *c = &e->sp.cache[k];
    const ms_arbiter_state *a = &s->arb[k];
    c->pair = a->pair; c->count = a->count; c->idle = a->idle;
    for (int i = 0; i < 2; ++i) { c->hash[i] = a->hash[i]; c->jn[i] = a->jn[i]; c->jt[i] = a->jt[i]; }
  }
}

/* Goal soft reset alone (Game._reset_positions, game.py:120-127), for the spawn fixtures. */
ORC_API void orc_env_soft_reset(orc_env *e) { spawn(e, e->mode); }

/* ---- batched helpers (tests, bench cpu_baseline) ---- */
ORC_API void orc_batch_reset(orc_env *envs, int n, const orc_params *P, const uint64_t *pcg, int mode,
                             float *obs) {
  for (int i = 0; i < n; ++i)
    orc_env_reset(&envs[i], P, pcg ? pcg + 4 * (size_t)i : NULL, mode, obs ? obs + (size_t)i * 264 : NULL);
}

ORC_API int orc_batch_step(orc_env *envs, int n, const orc_params *P, const float *act, float *obs,
                           double *rew, uint8_t *trunc, int8_t *goal, int32_t *score) {
  int bad = 0;
  for (int i = 0; i < n; ++i) {
    size_t k = (size_t)i;
    int rc = orc_env_step(&envs[i], P, act + 12 * k, obs ? obs + 264 * k : NULL, rew ? rew + 4 * k : NULL,
                          trunc ? trunc + 4 * k : NULL, goal ? goal + k : NULL, score ? score + 2 * k : NULL);
    if (rc) bad++;
  }
  return bad;
}

ORC_API void orc_batch_export(const orc_env *envs, int n, ms_env_state *out) {
  for (int i = 0; i < n; ++i) orc_env_export(&envs[i], &out[i]);
}
ORC_API void orc_batch_import(orc_env *envs, int n, const ms_env_state *in) {
  for (int i = 0; i < n; ++i) orc_env_import(&envs[i], &in[i]);
}
ORC_API void orc_batch_observe(const orc_env *envs, int n, const orc_params *P, float *frames) {
  for (int i = 0; i < n; ++i) orc_env_observe(&envs[i], P, frames + (size_t)i * 88);
}
ORC_API void orc_batch_positions(const orc_env *envs, int n, double *out) {
  for (int i = 0; i < n; ++i)
    for (int b = 0; b < 5; ++b) {
      out[(size_t)i * 10 + b * 2] = (double)envs[i].sp.body[b].px;
      out[(size_t)i * 10 + b * 2 + 1] = (double)envs[i].sp.body[b].py;
    }
}
ORC_API void orc_batch_rng(const orc_env *envs, int n, uint64_t *out) {
  for (int i = 0; i < n; ++i) {
    const orc_rng *g = &envs[i].rng;
    uint64_t *o = out + (size_t)i * 6;
    o[0] = g->state_hi; o[1] = g->state_lo; o[2] = g->inc_hi; o[3] = g->inc_lo;
    o[4] = (uint64_t)g->has_uint32; o[5] = g->uinteger;
  }
}
ORC_API void orc_batch_soft_reset(orc_env *envs, int n) {
  for (int i = 0; i < n; ++i) orc_env_soft_reset(&envs[i]);
}
/* contacts in each env's last physics step (instrumentation for kernel tuning) */
ORC_API void orc_batch_ncontacts(const orc_env *envs, int n, int32_t *out) {
  for (int i = 0; i < n; ++i) {
    int c = 0;
    for (int k = 0; k < envs[i].sp.n_arb; ++k) c += envs[i].sp.arb[k].count;
    out[i] = c;
  }
}
ORC_API unsigned long long orc_batch_overflow(const orc_env *envs, int n) {
  unsigned long long s = 0;
  for (int i = 0; i < n; ++i) s += envs[i].sp.overflow;
  return s;
}

/* ---- CPU baseline: the serial SyncMultiAgentVecEnv loop over env shards on T threads ---- */
typedef struct { orc_env *envs; int n, steps; const orc_params *P; uint64_t seed; } orc_job;

static float hash_action(uint64_t key) { /* splitmix64 -> uniform(-1, 1) fp32 */
  uint64_t z = key + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  z = z ^ (z >> 31);
  return (float)((double)(z >> 40) * (2.0 / 16777216.0) - 1.0);
}

static void *orc_job_run(void *arg) {
  orc_job *j = (orc_job *)arg;
  float act[12], obs[264]; double rew[4]; uint8_t tr[4]; int8_t g; int32_t sc[2];
  for (int t = 0; t < j->steps; ++t)
    for (int i = 0; i < j->n; ++i) {
      for (int k = 0; k < 12; ++k) act[k] = hash_action(j->seed ^ ((uint64_t)t << 32) ^ ((uint64_t)i * 12 + k));
      orc_env_step(&j->envs[i], j->P, act, obs, rew, tr, &g, sc);
    }
  return NULL;
}

/* Runs n_envs x n_steps env-steps on `threads` threads; returns wall seconds. */
ORC_API double orc_cpu_baseline(const orc_params *P, int n_envs, int n_steps, int threads, uint64_t seed) {
  orc_env *envs = (orc_env *)calloc((size_t)n_envs, sizeof(orc_env));
  if (!envs) return -1.0;
  for (int i = 0; i < n_envs; ++i) {
    uint64_t pcg[4] = {0x0123456789ABCDEFULL ^ (uint64_t)i, 0x0FEDCBA987654321ULL + (uint64_t)i,
                       0x5851F42D4C957F2DULL, ((uint64_t)i << 1) | 1u};
    orc_env_reset(&envs[i], P, pcg, MS_SPAWN_RANDOM, NULL);
  }
  if (threads < 1) threads = 1;
  if (threads > n_envs) threads = n_envs;
  pthread_t th[256]; orc_job jobs[256];
  if (threads > 256) threads = 256;
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  int per = (n_envs + threads - 1) / threads;
  int started = 0;
  for (int t = 0; t < threads; ++t) {
    int lo = t * per, hi = lo + per > n_envs ? n_envs : lo + per;
    if (lo >= hi) break;
    jobs[t].envs = envs + lo; jobs[t].n = hi - lo; jobs[t].steps = n_steps; jobs[t].P = P;
    jobs[t].seed = seed + (uint64_t)lo * 0x100000001ULL;
    pthread_create(&th[t], NULL, orc_job_run, &jobs[t]);
    started++;
  }
  for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  free(envs);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

ORC_API const char *orc_precision(void) { return ORC_NAME; }
