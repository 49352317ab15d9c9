// ms_device.h — device-side arithmetic of the MI355X soccer env step (gfx950, fp32).
//
// Every floating-point operation here is part of the parity contract with the fp32 CPU
// oracle (oracle/soccer_oracle.c, -DORC_F32): same operations, same order, no FMA
// contraction (-ffp-contract=off), IEEE division/sqrt (hipcc default), own sin/cos. Each
// function cites the reference code (or the Chipmunk2D routine behind pymunk) it restates.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/marl_soccer.h"

namespace ms {

// ------------------------------------------------------------------------------------------
// Parameters (computed on the host by ms_create, passed by value as a kernel argument)
// ------------------------------------------------------------------------------------------
struct Seg {
  float ax, ay, bx, by, nx, ny, r;
  float bb[4];
};

struct Params {
  float dt, slop, bias_coef;
  float m_inv[6], i_inv[6];  // agents 0..3, ball 4, static 5 (= 0)
  float agent_damp, ball_damp, vmax;
  float force_max, torque_max;
  float obs_vmax, obs_wmax;
  float e_aa, u_aa, e_ab, u_ab, e_aw, u_aw, e_ag, u_ag, e_bw, u_bw;
  float prox_mult, goal_mult, alive, goal_reward, concede_penalty, score_diff_mult;
  int max_steps, autoreset;
  int fast_div;  // obs_vmax, obs_wmax inside div_nr's divisor domain (host-checked)
  Seg seg[8];
};

// ------------------------------------------------------------------------------------------
// cpVect helpers (Chipmunk chipmunk_types.h / cpVect.h semantics)
// ------------------------------------------------------------------------------------------
// 2-vectors as a clang vector type: every x/y pair operation below is one packed fp32
// instruction (v_pk_add_f32 / v_pk_mul_f32, per-half negation as a source modifier). Each
// component is the same IEEE operation on the same operands as the scalar formula (no
// contraction: -ffp-contract=off), so results are bit-identical to the scalar restatement.
typedef float V2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ V2 v2(float x, float y) { return V2{x, y}; }
__device__ __forceinline__ V2 vadd(V2 a, V2 b) { return a + b; }
__device__ __forceinline__ V2 vsub(V2 a, V2 b) { return a - b; }
__device__ __forceinline__ V2 vneg(V2 a) { return -a; }
__device__ __forceinline__ V2 vmult(V2 a, float s) { return a * s; }
// c + a * s, each component one fused multiply-add (v_pk_fma_f32, one rounding): the solver's
// velocity updates. The fp32 oracle computes the same places with fmaf (soccer_oracle.c SMADD).
__device__ __forceinline__ V2 vmadd(V2 a, float s, V2 c) { return __builtin_elementwise_fma(a, V2{s, s}, c); }
// a.x * b.x + a.y * b.y
__device__ __forceinline__ float vdot(V2 a, V2 b) { const V2 p = a * b; return p.x + p.y; }
// a.x * b.y - a.y * b.x
__device__ __forceinline__ float vcross(V2 a, V2 b) { const V2 p = a * b.yx; return p.x - p.y; }
__device__ __forceinline__ V2 vperp(V2 a) { return v2(-a.y, a.x); }
// (a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x) with the outer add fused (solver impulses only;
// the fp32 oracle's vrotate is the same SMADD form). The low product's sign comes from its
// multiplicand, (-a.y) * b.y = -(a.y * b.y) exactly, which is off the solver's dependency chain (a
// is the contact normal), instead of a multiply of the product by (-1, 1) on it
__device__ __forceinline__ V2 vrotate(V2 a, V2 b) {
  return __builtin_elementwise_fma(V2{a.x, a.x}, b, V2{-a.y, a.y} * b.yx);
}
__device__ __forceinline__ float vlengthsq(V2 a) { return vdot(a, a); }
__device__ __forceinline__ float fmaxr(float a, float b) { return (a > b) ? a : b; }  // cpfmax
__device__ __forceinline__ float fminr(float a, float b) { return (a < b) ? a : b; }  // cpfmin
__device__ __forceinline__ float fclamp(float f, float lo, float hi) { return fminr(fmaxr(f, lo), hi); }
// fclamp(f, -M, M) (the friction clamp) by one v_med3_f32 instead of two compare-select pairs on
// the solver's dependency chain: for M > 0 the median of (f, -M, M) is fclamp's value (bit for
// bit for finite f: -M < f < M returns f itself, else the bound it crossed); for M <= 0 (or NaN)
// fclamp returns M whatever f is (fmaxr(f, -M) >= -M >= M, then fminr(., M) = M, signed zeros
// included)
__device__ __forceinline__ float fclamp_sym(float f, float M) {
  const float m = __builtin_amdgcn_fmed3f(f, -M, M);
  return M > 0.0f ? m : M;
}
__device__ __forceinline__ float fclamp01(float f) { return fmaxr(0.0f, fminr(f, 1.0f)); }
__device__ __forceinline__ V2 vlerp(V2 a, V2 b, float t) { return vadd(vmult(a, 1.0f - t), vmult(b, t)); }

// cpCollision.c ClosestT / LerpT
__device__ __forceinline__ float closest_t(V2 a, V2 b) {
  V2 delta = vsub(b, a);
  return -fclamp(vdot(delta, vadd(a, b)) / vlengthsq(delta), -1.0f, 1.0f);
}
__device__ __forceinline__ V2 lerp_t(V2 a, V2 b, float t) {
  float ht = 0.5f * t;
  return vadd(vmult(a, 0.5f - ht), vmult(b, 0.5f + ht));
}

// ------------------------------------------------------------------------------------------
// fp32 trigonometry contract: Cody-Waite pi/2 reduction (parts of <= 12 significant bits)
// + cephes sinf/cosf polynomials. Replaces Chipmunk's cpvforangle (cos, sin) and the
// atan2(sin, cos)/pi angle wrap of game.py:272-274.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void sincos_contract(float x, float* s_out, float* c_out) {
  if (!(x == x) || fabsf(x) > 1.0e30f) {
    *s_out = __builtin_nanf("");
    *c_out = __builtin_nanf("");
    return;
  }
  float kf = rintf(x * 0.636619746685028076171875f);
  kf = kf > 1073741824.0f ? 1073741824.0f : kf;
  kf = kf < -1073741824.0f ? -1073741824.0f : kf;
  int q = (int)kf;
  float r = ((x - kf * 1.5703125f) - kf * 4.838705062866211e-4f) - kf * -4.371138828673793e-8f;
  float z = r * r;
  float sr = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * r + r;
  float cr = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z -
             0.5f * z + 1.0f;
  switch (q & 3) {
    case 0: *s_out = sr; *c_out = cr; break;
    case 1: *s_out = cr; *c_out = -sr; break;
    case 2: *s_out = -sr; *c_out = -cr; break;
    default: *s_out = -cr; *c_out = sr; break;
  }
}

// ------------------------------------------------------------------------------------------
// Reduced-range IEEE division and square root. The compiler's correctly rounded fp32 division
// is v_div_scale x2, v_rcp, Newton refinement, v_div_fmas, v_div_fixup; for a positive normal
// divisor d in [2^-26, 2^13] and a numerator n = 0 or 2^-100 <= |n| <= 2^30, div_scale scales
// nothing, div_fmas is a plain fma and div_fixup is the identity, so the sequence below returns
// the same bits as n / d (and the reciprocal refinement is shared by every division by d).
// Likewise sqrt_nr is the compiler's sqrtf without the tiny-input rescale and the zero/inf
// class fix-up, identical for x in [2^-90, 2^126]. Both were checked on the MI355X against
// IEEE over 1.7e10 random operands of those domains with no difference; callers guard their
// inputs (frame_inputs_in_range) and take the IEEE path otherwise.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float rcp_nr(float d) {
  const float r = __builtin_amdgcn_rcpf(d);
  const float e = __builtin_fmaf(-d, r, 1.0f);
  return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ float div_nr(float n, float d, float r) {
  float q = n * r;
  float e = __builtin_fmaf(-d, q, n);
  q = __builtin_fmaf(e, r, q);
  e = __builtin_fmaf(-d, q, n);
  const float res = __builtin_fmaf(e, r, q);
  return n == 0.0f ? n : res;  // keeps the sign of a zero numerator
}
// div_nr of both components of a pair: the same operations per component as packed fp32
// (v_pk_mul_f32 / v_pk_fma_f32)
__device__ __forceinline__ V2 div_nr2(V2 n, float d, float r) {
  const V2 nd = V2{-d, -d}, rv = V2{r, r};
  V2 q = n * rv;
  V2 e = __builtin_elementwise_fma(nd, q, n);
  q = __builtin_elementwise_fma(e, rv, q);
  e = __builtin_elementwise_fma(nd, q, n);
  V2 res = __builtin_elementwise_fma(e, rv, q);
  res.x = n.x == 0.0f ? n.x : res.x;
  res.y = n.y == 0.0f ? n.y : res.y;
  return res;
}
// div_nr for a numerator that is never -0: a +0 numerator gives +0 through the Newton steps
// themselves (fma(-d, +0, +0) = +0 for d > 0), so the zero select is not needed
__device__ __forceinline__ float div_nr_nonneg(float n, float d, float r) {
  float q = n * r;
  float e = __builtin_fmaf(-d, q, n);
  q = __builtin_fmaf(e, r, q);
  e = __builtin_fmaf(-d, q, n);
  return __builtin_fmaf(e, r, q);
}
// One-residual quotients for the frame arithmetic's fixed divisors: 1000 (magnitudes), pi (angle_obs)
// and the default obs_vmax 200 / obs_wmax 10. For d one of those and r = rcp_nr(d), q0 = n r corrected
// once, fma(fma(-d, q0, n), r, q0), equals the IEEE n / d for EVERY fp32 numerator of either sign in
// [2^-100, 2^32) (exhaustive check on the MI355X: tools/div_check.hip, profiles/r05s/div_check.txt),
// which holds every numerator the fast paths admit; a -0 numerator is kept by the select as in div_nr.
// obs_div takes this path only where the divisor is one of those constants at compile time (the
// specialised kernels: ms_config_specialised 1 and 2), div_nr otherwise.
#ifndef MS_DIV_ONESTEP
#define MS_DIV_ONESTEP 1
#endif
__device__ __forceinline__ float div_k(float n, float d, float r) {
  const float q = n * r;
  const float e = __builtin_fmaf(-d, q, n);
  const float res = __builtin_fmaf(e, r, q);
  return n == 0.0f ? n : res;
}
__device__ __forceinline__ float div_k_nonneg(float n, float d, float r) {  // n never -0
  const float q = n * r;
  return __builtin_fmaf(__builtin_fmaf(-d, q, n), r, q);
}
__device__ __forceinline__ bool div_k_ok(float d) {
  return MS_DIV_ONESTEP && __builtin_constant_p(d) && (d == 200.0f || d == 10.0f || d == 1000.0f);
}
__device__ __forceinline__ float obs_div(float n, float d) {
  if (div_k_ok(d)) return div_k(n, d, rcp_nr(d));
  return div_nr(n, d, rcp_nr(d));
}
__device__ __forceinline__ float sqrt_nr(float x) {
  float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
  const float rm = __builtin_fmaf(-sm, s, x), rp = __builtin_fmaf(-sp, s, x);
  s = rm <= 0.0f ? sm : s;
  s = rp > 0.0f ? sp : s;
  return s;
}

template <bool FAST = false>
__device__ __forceinline__ float angle_obs(float a) {
  float k = rintf(a * 0.15915493667125702f);
  float w = (a - k * 6.28125f) - k * 0.0019353071693331003f;
  if constexpr (FAST) {
    if (MS_DIV_ONESTEP) return div_k(w, 3.1415927410125732f, rcp_nr(3.1415927410125732f));
    return div_nr(w, 3.1415927410125732f, rcp_nr(3.1415927410125732f));
  }
  return w / 3.1415927410125732f;
}

// ------------------------------------------------------------------------------------------
// Geometry
// ------------------------------------------------------------------------------------------
// World box of an agent: cpBoxShapeNew(body, 30, 30, 0) after cpPolyShapeCacheData.
// plane i: v[i] = vertex i, n[i] = outward normal of edge v[i-1] -> v[i].
struct Box {
  V2 v[4], n[4];
  float bb[4];
};

__device__ __forceinline__ void box_world(float px, float py, float c, float s, Box& o) {
  const float LX[4] = {15.0f, 15.0f, -15.0f, -15.0f};
  const float LY[4] = {-15.0f, 15.0f, 15.0f, -15.0f};
#pragma unroll
  for (int i = 0; i < 4; ++i) o.v[i] = v2((c * LX[i] + (-s) * LY[i]) + px, (s * LX[i] + c * LY[i]) + py);
  o.n[0] = v2(s, -c);
  o.n[1] = v2(c, s);
  o.n[2] = v2(-s, c);
  o.n[3] = v2(-c, -s);
  float l = o.v[0].x, r = o.v[0].x, bt = o.v[0].y, t = o.v[0].y;
#pragma unroll
  for (int i = 1; i < 4; ++i) {
    l = fminr(l, o.v[i].x);
    r = fmaxr(r, o.v[i].x);
    bt = fminr(bt, o.v[i].y);
    t = fmaxr(t, o.v[i].y);
  }
  o.bb[0] = l; o.bb[1] = bt; o.bb[2] = r; o.bb[3] = t;
}

__device__ __forceinline__ bool bb_intersects(const float* a, const float* b) {
  return a[0] <= b[2] && b[0] <= a[2] && a[1] <= b[3] && b[1] <= a[3];
}

// Narrowphase result: up to 2 contacts with absolute points (cpCollisionInfo)
struct Col {
  int count;
  V2 n;
  V2 p1[2], p2[2];
  int hash[2];
};

__device__ __forceinline__ void push_contact(Col& col, V2 p1, V2 p2, int hash) {
  if (col.count == 0) {
    col.p1[0] = p1; col.p2[0] = p2; col.hash[0] = hash;
  } else {
    col.p1[1] = p1; col.p2[1] = p2; col.hash[1] = hash;
  }
  col.count++;
}

struct Edge {
  V2 a, b;
  int ha, hb;
  float r;
};

// SupportEdgeForPoly (cpCollision.c)
__device__ __forceinline__ Edge support_edge_box(const Box& bx, V2 n) {
  int i1 = 0;
  float mx = -__builtin_inff();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float d = vdot(bx.v[i], n);
    if (d > mx) { mx = d; i1 = i; }
  }
  int i0 = (i1 + 3) & 3, i2 = (i1 + 1) & 3;
  // select by index without dynamic register indexing
  V2 v0 = bx.v[0], v1 = bx.v[0], v2_ = bx.v[0], n1 = bx.n[0], n2 = bx.n[0];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i == i0) v0 = bx.v[i];
    if (i == i1) { v1 = bx.v[i]; n1 = bx.n[i]; }
    if (i == i2) { v2_ = bx.v[i]; n2 = bx.n[i]; }
  }
  Edge e;
  e.r = 0.0f;
  if (vdot(n, n1) > vdot(n, n2)) {
    e.a = v0; e.ha = i0; e.b = v1; e.hb = i1;
  } else {
    e.a = v1; e.ha = i1; e.b = v2_; e.hb = i2;
  }
  return e;
}

// SupportEdgeForSegment (cpCollision.c)
__device__ __forceinline__ Edge support_edge_seg(const Seg& s, V2 n) {
  Edge e;
  e.r = s.r;
  if (vdot(v2(s.nx, s.ny), n) > 0.0f) {
    e.a = v2(s.ax, s.ay); e.ha = 0; e.b = v2(s.bx, s.by); e.hb = 1;
  } else {
    e.a = v2(s.bx, s.by); e.ha = 1; e.b = v2(s.ax, s.ay); e.hb = 0;
  }
  return e;
}

#define MS_FEATURE_HASH(h1, h2) (0x10 | ((h1) << 2) | (h2))

// ContactPoints (cpCollision.c)
__device__ __forceinline__ void contact_points(const Edge& e1, const Edge& e2, float d, V2 n, Col& col) {
  float mindist = e1.r + e2.r;
  if (!(d <= mindist)) return;
  col.n = n;
  float d_e1_a = vcross(e1.a, n), d_e1_b = vcross(e1.b, n);
  float d_e2_a = vcross(e2.a, n), d_e2_b = vcross(e2.b, n);
  float e1_denom = 1.0f / (d_e1_b - d_e1_a + 1.17549435082228750797e-38f);
  float e2_denom = 1.0f / (d_e2_b - d_e2_a + 1.17549435082228750797e-38f);
  {
    V2 p1 = vadd(vmult(n, e1.r), vlerp(e1.a, e1.b, fclamp01((d_e2_b - d_e1_a) * e1_denom)));
    V2 p2 = vadd(vmult(n, -e2.r), vlerp(e2.a, e2.b, fclamp01((d_e1_a - d_e2_a) * e2_denom)));
    float dist = vdot(vsub(p2, p1), n);
    if (dist <= 0.0f) push_contact(col, p1, p2, MS_FEATURE_HASH(e1.ha, e2.hb));
  }
  {
    V2 p1 = vadd(vmult(n, e1.r), vlerp(e1.a, e1.b, fclamp01((d_e2_a - d_e1_a) * e1_denom)));
    V2 p2 = vadd(vmult(n, -e2.r), vlerp(e2.a, e2.b, fclamp01((d_e1_b - d_e2_a) * e2_denom)));
    float dist = vdot(vsub(p2, p1), n);
    if (dist <= 0.0f) push_contact(col, p1, p2, MS_FEATURE_HASH(e1.hb, e2.ha));
  }
}

// CircleToSegment (cpCollision.c): ball (a) vs wall (b)
__device__ __forceinline__ void col_circle_seg(V2 center, float cr, const Seg& s, Col& col) {
  V2 sa = v2(s.ax, s.ay), sb = v2(s.bx, s.by);
  V2 seg_delta = vsub(sb, sa);
  float ct = fclamp01(vdot(seg_delta, vsub(center, sa)) / vlengthsq(seg_delta));
  V2 closest = vadd(sa, vmult(seg_delta, ct));
  float mindist = cr + s.r;
  V2 delta = vsub(closest, center);
  // An interior closest point is the centre's foot on the segment's line: closest - centre =
  // n_s (n_s . (a - centre)), the same vector without the ~ulp(|b - a|) tangential residue that
  // a + (b - a) t - centre keeps in fp32 (6e-5 px on a 780-px wall tilts the normal by 6e-6 and
  // a squeezed ball's ~2,000 impulse with it)
  if (ct > 0.0f && ct < 1.0f) {
    const V2 sn = v2(s.nx, s.ny);
    delta = vmult(sn, vdot(sn, vsub(sa, center)));
    closest = vadd(center, delta);
  }
  float distsq = vlengthsq(delta);
  if (distsq < mindist * mindist) {
    float dist = sqrtf(distsq);
    V2 n = (dist != 0.0f) ? vmult(delta, 1.0f / dist) : v2(s.nx, s.ny);
    col.n = n;
    push_contact(col, vadd(center, vmult(n, cr)), vadd(closest, vmult(n, -s.r)), 0);
  }
}

// CircleToPoly restated analytically: ball (a) vs agent box (b).
__device__ __forceinline__ void col_circle_box(V2 c, float cr, const Box& bx, Col& col) {
  int fi = 0;
  float smax = -__builtin_inff();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float s = vdot(bx.n[i], c) - vdot(bx.n[i], bx.v[i]);
    if (s > smax) { smax = s; fi = i; }
  }
  if (!(smax <= cr)) return;
  V2 n, pb;
  float d;
  if (smax <= 0.0f) {
    V2 v0 = bx.v[3], v1 = bx.v[0], fn = bx.n[0];
#pragma unroll
    for (int i = 1; i < 4; ++i)
      if (i == fi) { v0 = bx.v[i - 1]; v1 = bx.v[i]; fn = bx.n[i]; }
    float t = closest_t(vsub(v0, c), vsub(v1, c));
    pb = lerp_t(v0, v1, t);
    n = vneg(fn);
    d = smax;
  } else {
    float best = __builtin_inff(), tb = 0.0f;
    V2 fn = bx.n[0];
    pb = v2(0.0f, 0.0f);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      V2 v0 = bx.v[(i + 3) & 3], v1 = bx.v[i];
      V2 a = vsub(v0, c), b = vsub(v1, c);
      float t = closest_t(a, b);
      V2 p = lerp_t(a, b, t);
      float d2 = vlengthsq(p);
      if (d2 < best) { best = d2; pb = lerp_t(v0, v1, t); fn = bx.n[i]; tb = t; }
    }
    V2 p = vsub(pb, c);
    if (tb > -1.0f && tb < 1.0f) {
      n = vneg(fn);
      d = vdot(n, p);
    } else {
      d = sqrtf(vlengthsq(p));
      n = vmult(p, 1.0f / (d + 1.17549435082228750797e-38f));
    }
  }
  if (d <= cr) {
    col.n = n;
    push_contact(col, vadd(c, vmult(n, cr)), pb, 0);
  }
}

// SegmentToPoly restated: wall (a) vs agent box (b)
__device__ __forceinline__ void col_seg_box(const Seg& s, const Box& bx, Col& col) {
  V2 sa = v2(s.ax, s.ay), sb = v2(s.bx, s.by), sn = v2(s.nx, s.ny);
  float smax = -__builtin_inff();
  V2 axis = v2(0.0f, 0.0f);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    V2 an = k == 0 ? sn : vneg(sn);
    float m = __builtin_inff();
#pragma unroll
    for (int j = 0; j < 4; ++j) m = fminr(m, vdot(an, bx.v[j]));
    float sep = m - vdot(an, sa);
    if (sep > smax) { smax = sep; axis = an; }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float m = fminr(vdot(bx.n[i], sa), vdot(bx.n[i], sb));
    float sep = m - vdot(bx.n[i], bx.v[i]);
    if (sep > smax) { smax = sep; axis = vneg(bx.n[i]); }
  }
  if (!(smax <= s.r)) return;
  V2 n;
  float d;
  if (smax <= 0.0f) {
    n = axis;
    d = smax;
  } else {
    float best = __builtin_inff();
    V2 pa = v2(0.0f, 0.0f), pb = v2(0.0f, 0.0f), fn = v2(0.0f, 0.0f);
    int kind = 0;
    // The sequential minimum below keeps the first candidate of the smallest d2 (endpoint
    // candidates first, then box vertices). The vertex candidates are evaluated first here;
    // an endpoint whose distance to the box's bounding box exceeds the best vertex distance
    // by more than 0.5 (far above the fp32 rounding of any candidate's d2) cannot be that
    // minimum, so its four edge candidates are skipped. Same winner, same bits.
    float bestV = __builtin_inff();
    V2 paV = pa, pbV = pb, fnV = fn;
    int kindV = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      V2 a = vsub(sa, bx.v[j]), b = vsub(sb, bx.v[j]);
      float t = closest_t(a, b);
      V2 p = lerp_t(a, b, t);
      float d2 = vlengthsq(p);
      if (d2 < bestV) {
        bestV = d2; paV = lerp_t(sa, sb, t); pbV = bx.v[j];
        if (t > -1.0f && t < 1.0f) {
          kindV = 1;
          fnV = (vdot(sn, vsub(bx.v[j], sa)) > 0.0f) ? sn : vneg(sn);
        } else kindV = 0;
      }
    }
    const float reach = __builtin_amdgcn_sqrtf(bestV) + 0.5f;
    bool need[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const V2 e = k == 0 ? sa : sb;
      const float dx = fmaxf(fmaxf(bx.bb[0] - e.x, e.x - bx.bb[2]), 0.0f);
      const float dy = fmaxf(fmaxf(bx.bb[1] - e.y, e.y - bx.bb[3]), 0.0f);
      need[k] = !(dx * dx + dy * dy > reach * reach);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (!need[k]) continue;
      V2 e = k == 0 ? sa : sb;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        V2 v0 = bx.v[(i + 3) & 3], v1 = bx.v[i];
        V2 a = vsub(v0, e), b = vsub(v1, e);
        float t = closest_t(a, b);
        V2 p = lerp_t(a, b, t);
        float d2 = vlengthsq(p);
        if (d2 < best) {
          best = d2; pa = e; pb = lerp_t(v0, v1, t);
          if (t > -1.0f && t < 1.0f) { kind = 1; fn = vneg(bx.n[i]); } else kind = 0;
        }
      }
    }
    if (bestV < best) { best = bestV; pa = paV; pb = pbV; fn = fnV; kind = kindV; }
    V2 p = vsub(pb, pa);
    if (kind) {
      n = fn;
      d = vdot(n, p);
    } else {
      d = sqrtf(vlengthsq(p));
      n = vmult(p, 1.0f / (d + 1.17549435082228750797e-38f));
    }
  }
  if (d - s.r - 0.0f <= 0.0f) contact_points(support_edge_seg(s, n), support_edge_box(bx, vneg(n)), d, n, col);
}

// PolyToPoly restated: SAT over both boxes' face normals. A = lower agent index.
__device__ __forceinline__ void col_box_box(const Box& A, const Box& B, Col& col) {
  float smax = -__builtin_inff();
  V2 axis = v2(0.0f, 0.0f);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float m = __builtin_inff();
#pragma unroll
    for (int j = 0; j < 4; ++j) m = fminr(m, vdot(A.n[i], B.v[j]));
    float sep = m - vdot(A.n[i], A.v[i]);
    if (sep > smax) { smax = sep; axis = A.n[i]; }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float m = __builtin_inff();
#pragma unroll
    for (int j = 0; j < 4; ++j) m = fminr(m, vdot(B.n[i], A.v[j]));
    float sep = m - vdot(B.n[i], B.v[i]);
    if (sep > smax) { smax = sep; axis = vneg(B.n[i]); }
  }
  if (!(smax - 0.0f - 0.0f <= 0.0f)) return;
  contact_points(support_edge_box(A, axis), support_edge_box(B, vneg(axis)), smax, axis, col);
}

// ------------------------------------------------------------------------------------------
// numpy PCG64 (XSL-RR 128/64), Generator.uniform and integers(0, 4) — game.py:17, 81-85
// ------------------------------------------------------------------------------------------
struct Rng {
  uint64_t shi, slo, ihi, ilo;
  uint32_t has32, u32;
};

__device__ __forceinline__ uint64_t pcg_next64(Rng& g) {
  const uint64_t MH = 0x2360ED051FC65DA4ULL, ML = 0x4385DF649FCCF645ULL;
  uint64_t lo = g.slo * ML;
  uint64_t hi = __umul64hi(g.slo, ML) + g.shi * ML + g.slo * MH;
  uint64_t nlo = lo + g.ilo;
  uint64_t nhi = hi + g.ihi + (nlo < lo ? 1ULL : 0ULL);
  g.slo = nlo;
  g.shi = nhi;
  uint64_t x = nhi ^ nlo;
  unsigned rot = (unsigned)(nhi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}
__device__ __forceinline__ uint32_t pcg_next32(Rng& g) {
  if (g.has32) { g.has32 = 0; return g.u32; }
  uint64_t nx = pcg_next64(g);
  g.has32 = 1;
  g.u32 = (uint32_t)(nx >> 32);
  return (uint32_t)(nx & 0xffffffffu);
}
__device__ __forceinline__ double rng_uniform(Rng& g, double lo, double hi) {
  double u = (double)(pcg_next64(g) >> 11) * (1.0 / 9007199254740992.0);
  return lo + (hi - lo) * u;
}
__device__ __forceinline__ int rng_int4(Rng& g) {
  uint64_t m = (uint64_t)pcg_next32(g) * 4u;
  return (int)(m >> 32);
}

// Spawn modes: _apply_fixed_positions / _apply_random_positions /
// _apply_full_random_positions (game.py:129-249). Writes positions (fp32-rounded doubles).
__device__ __forceinline__ void spawn_positions(Rng& g, int mode, float px[5], float py[5]) {
  double x[5], y[5];
  if (mode == MS_SPAWN_FIXED) {
    x[0] = 800 * 0.25; y[0] = 600 * 0.33; x[1] = 800 * 0.25; y[1] = 600 * 0.66;
    x[2] = 800 * 0.75; y[2] = 600 * 0.33; x[3] = 800 * 0.75; y[3] = 600 * 0.66;
    x[4] = 400.0; y[4] = 300.0;
  } else if (mode == MS_SPAWN_RANDOM) {
    x[0] = rng_uniform(g, 30.0, 380.0); y[0] = rng_uniform(g, 30.0, 570.0);
    x[1] = rng_uniform(g, 30.0, 380.0); y[1] = rng_uniform(g, 30.0, 570.0);
    x[2] = rng_uniform(g, 420.0, 770.0); y[2] = rng_uniform(g, 30.0, 570.0);
    x[3] = rng_uniform(g, 420.0, 770.0); y[3] = rng_uniform(g, 30.0, 570.0);
    x[4] = 400.0 + rng_uniform(g, -40.0, 40.0);
    y[4] = 300.0 + rng_uniform(g, -40.0, 40.0);
  } else {
    double u0 = rng_uniform(g, 0.0, 1.0);
    if (u0 < 0.75) {
      int c1 = rng_int4(g), c2 = rng_int4(g);
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        int c = k == 0 ? c1 : c2;
        bool left = c == 0 || c == 1, top = c == 0 || c == 2;
        double cx = left ? 18.0 : 782.0, cy = top ? 582.0 : 18.0;
        double jx = rng_uniform(g, -5.0, 5.0);
        double jy = rng_uniform(g, -5.0, 5.0);
        x[k] = cx + jx;
        y[k] = cy + jy;
      }
    } else {
      x[0] = rng_uniform(g, 30.0, 770.0); y[0] = rng_uniform(g, 30.0, 570.0);
      x[1] = rng_uniform(g, 30.0, 770.0); y[1] = rng_uniform(g, 30.0, 570.0);
    }
    x[2] = rng_uniform(g, 30.0, 770.0); y[2] = rng_uniform(g, 30.0, 570.0);
    x[3] = rng_uniform(g, 30.0, 770.0); y[3] = rng_uniform(g, 30.0, 570.0);
    x[4] = rng_uniform(g, 30.0, 770.0); y[4] = rng_uniform(g, 30.0, 570.0);
  }
#pragma unroll
  for (int b = 0; b < 5; ++b) {
    px[b] = (float)x[b];
    py[b] = (float)y[b];
  }
}

// ------------------------------------------------------------------------------------------
// Observations: Game._get_observations (game.py:258-322) -> fp32 (soccer_env.py:131)
// ------------------------------------------------------------------------------------------
template <bool FAST = false>
__device__ __forceinline__ void unit_mag(float dx, float dy, float* o) {
  if constexpr (FAST) {
    // x and y as one packed pair: d*d, the two quotients' Newton steps (div_nr per component)
    const V2 d = v2(dx, dy);
    const V2 d2 = d * d;
    float mag = sqrt_nr(d2.x + d2.y);
    const float r = rcp_nr(mag);
    const bool big = mag > 1e-8f;
    const V2 q = div_nr2(d, mag, r);
    o[0] = big ? q.x : 0.0f;
    o[1] = big ? q.y : 0.0f;
    mag = big ? mag : 0.0f;
    o[2] = MS_DIV_ONESTEP ? div_k_nonneg(mag, 1000.0f, rcp_nr(1000.0f)) : div_nr_nonneg(mag, 1000.0f, rcp_nr(1000.0f));  // mag >= +0
    return;
  }
  float mag = sqrtf(dx * dx + dy * dy);
  if (mag > 1e-8f) {
    o[0] = dx / mag;
    o[1] = dy / mag;
  } else {
    o[0] = 0.0f;
    o[1] = 0.0f;
    mag = 0.0f;
  }
  o[2] = mag / 1000.0f;  // field diagonal hypot(800, 600)
}

// unit_mag<true> of two vectors at once, for numerators that are never -0: the lane-pair kernel's fast
// path requires every position >= +0 (psnap_in_range tests the sign), and each numerator is a position
// or a positive goal coordinate minus a position, which is -0 only for (-0) - (+0). A +0 numerator
// leaves the Newton steps at +0 (fma(-d, +0, +0) = +0 for d > 0), so div_nr2's zero selects are not
// needed. The per-component operations are unit_mag<true>'s, the two vectors' scalar steps (squares,
// sqrt_nr's residuals, rcp_nr's refinement, the magnitude / 1000) paired as packed fp32.
__device__ __forceinline__ V2 div_nr2_pos(V2 n, float d, float r) {
  const V2 nd = V2{-d, -d}, rv = V2{r, r};
  V2 q = n * rv;
  V2 e = __builtin_elementwise_fma(nd, q, n);
  q = __builtin_elementwise_fma(e, rv, q);
  e = __builtin_elementwise_fma(nd, q, n);
  return __builtin_elementwise_fma(e, rv, q);
}
// div_k_nonneg of both components as packed fp32 (the magnitudes / 1000 of unit_mag2_pos); the same
// operations per component, checked with the scalar forms by tools/div_check.hip
__device__ __forceinline__ V2 div_k2_nonneg(V2 n, float d, float r) {
  const V2 q = n * V2{r, r};
  return __builtin_elementwise_fma(__builtin_elementwise_fma(V2{-d, -d}, q, n), V2{r, r}, q);
}
__device__ __forceinline__ void unit_mag_pos(float dx, float dy, float* o);
__device__ __forceinline__ void unit_mag2_pos(float ax, float ay, float bx, float by, float* oa, float* ob) {
  const V2 X = v2(ax, bx), Y = v2(ay, by);
  const V2 s2 = X * X + Y * Y;
  const V2 S = v2(__builtin_amdgcn_sqrtf(s2.x), __builtin_amdgcn_sqrtf(s2.y));
  const V2 SM = v2(__uint_as_float(__float_as_uint(S.x) - 1u), __uint_as_float(__float_as_uint(S.y) - 1u));
  const V2 SP = v2(__uint_as_float(__float_as_uint(S.x) + 1u), __uint_as_float(__float_as_uint(S.y) + 1u));
  const V2 RM = __builtin_elementwise_fma(-SM, S, s2), RP = __builtin_elementwise_fma(-SP, S, s2);
  V2 M;
  M.x = RM.x <= 0.0f ? SM.x : S.x;
  M.x = RP.x > 0.0f ? SP.x : M.x;
  M.y = RM.y <= 0.0f ? SM.y : S.y;
  M.y = RP.y > 0.0f ? SP.y : M.y;
  const V2 R0 = v2(__builtin_amdgcn_rcpf(M.x), __builtin_amdgcn_rcpf(M.y));
  const V2 E = __builtin_elementwise_fma(-M, R0, V2{1.0f, 1.0f});
  const V2 R = __builtin_elementwise_fma(E, R0, R0);
  const bool biga = M.x > 1e-8f, bigb = M.y > 1e-8f;
  const V2 qa = div_nr2_pos(v2(ax, ay), M.x, R.x), qb = div_nr2_pos(v2(bx, by), M.y, R.y);
  oa[0] = biga ? qa.x : 0.0f;
  oa[1] = biga ? qa.y : 0.0f;
  ob[0] = bigb ? qb.x : 0.0f;
  ob[1] = bigb ? qb.y : 0.0f;
  const V2 N = v2(biga ? M.x : 0.0f, bigb ? M.y : 0.0f);  // >= +0: div_nr_nonneg, paired
  const float r1k = rcp_nr(1000.0f);
  V2 qm;
  if (MS_DIV_ONESTEP) {
    qm = div_k2_nonneg(N, 1000.0f, r1k);
  } else {
    qm = div_nr2_pos(N, 1000.0f, r1k);
  }
  oa[2] = qm.x;
  ob[2] = qm.y;
}
// the same for one vector
__device__ __forceinline__ void unit_mag_pos(float dx, float dy, float* o) {
  const V2 d = v2(dx, dy);
  const V2 d2 = d * d;
  float mag = sqrt_nr(d2.x + d2.y);
  const float r = rcp_nr(mag);
  const bool big = mag > 1e-8f;
  const V2 q = div_nr2_pos(d, mag, r);
  o[0] = big ? q.x : 0.0f;
  o[1] = big ? q.y : 0.0f;
  mag = big ? mag : 0.0f;
  o[2] = MS_DIV_ONESTEP ? div_k_nonneg(mag, 1000.0f, rcp_nr(1000.0f)) : div_nr_nonneg(mag, 1000.0f, rcp_nr(1000.0f));
}

// frame of agent i (static), o[22]
template <int I>
__device__ __forceinline__ void agent_frame(const Params& P, const float px[5], const float py[5],
                                            const float vx[5], const float vy[5], const float ang[4],
                                            const float w[5], float* o) {
  constexpr int TEAM = I == 0 ? 1 : (I == 1 ? 0 : (I == 2 ? 3 : 2));
  constexpr int O1 = I < 2 ? 2 : 0, O2 = I < 2 ? 3 : 1;
  o[0] = vx[I] / P.obs_vmax;
  o[1] = vy[I] / P.obs_vmax;
  o[2] = angle_obs(ang[I]);
  o[3] = w[I] / P.obs_wmax;
  unit_mag(px[TEAM] - px[I], py[TEAM] - py[I], o + 4);
  unit_mag(px[O1] - px[I], py[O1] - py[I], o + 7);
  unit_mag(px[O2] - px[I], py[O2] - py[I], o + 10);
  unit_mag(px[4] - px[I], py[4] - py[I], o + 13);
  const float own_x = I < 2 ? 10.0f : 790.0f, opp_x = I < 2 ? 790.0f : 10.0f;
  unit_mag(own_x - px[I], 300.0f - py[I], o + 16);
  unit_mag(opp_x - px[I], 300.0f - py[I], o + 19);
}

// ------------------------------------------------------------------------------------------
// Rewards: _update_reward_state + _calculate_rewards + terminal override
// (game.py:251-256, 324-375, 424-433); distance improvements in difference-of-squares form.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float dist_improvement(float a0x, float a0y, float b0x, float b0y, float a1x,
                                                  float a1y, float b1x, float b1y) {
  float px = a0x - b0x, py = a0y - b0y;
  float cx = a1x - b1x, cy = a1y - b1y;
  float dax = a1x - a0x, day = a1y - a0y;
  float dbx = b1x - b0x, dby = b1y - b0y;
  float num = (dbx - dax) * (px + cx) + (dby - day) * (py + cy);
  float den = sqrtf(px * px + py * py) + sqrtf(cx * cx + cy * cy);
  return den > 0.0f ? num / den : 0.0f;
}

__device__ __forceinline__ float blue_reward(const Params& P, const float pvx[5], const float pvy[5],
                                             const float cux[5], const float cuy[5], int goal, bool terminal,
                                             int score_blue, int score_red) {
  if (terminal) return P.score_diff_mult * (float)(score_blue - score_red);
  float r = 0.0f;
  if (P.prox_mult != 0.0f) {
    float imp = dist_improvement(pvx[0], pvy[0], pvx[4], pvy[4], cux[0], cuy[0], cux[4], cuy[4]) +
                dist_improvement(pvx[1], pvy[1], pvx[4], pvy[4], cux[1], cuy[1], cux[4], cuy[4]);
    r = r + P.prox_mult * imp;
  }
  float g = dist_improvement(pvx[4], pvy[4], 790.0f, 300.0f, cux[4], cuy[4], 790.0f, 300.0f);
  r = r + g * P.goal_mult;
  if (goal == 1) r = r + P.goal_reward;
  else if (goal == 2) r = r - P.concede_penalty;
  r = r - P.alive;
  return r;
}

}  // namespace ms
