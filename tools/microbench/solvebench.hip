// Diagnostic (not product): cycles per contact solve of the lane-group serial path, built from the
// kernel's own device functions. Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950
// -o solvebench solvebench.hip ; run on the GPU box: ./solvebench (small-shard floor)
// scratch microbenchmark (not product): cycles per contact solve of the lane-group serial path
#include "../../marl-soccer_amd/csrc/ms_env.hip"
using namespace grp;
// scalar restatement (same operations, no packed pairs) for a latency comparison
__device__ __forceinline__ void solve_hs(const Params& P, HSlot& c, float4* rec) {
  const int ba = CS_BA(c.m), bb = CS_BB(c.m);
  const float ma = body_minv(P, ba), ia = body_iinv(P, ba), mb = body_b_minv(P, bb), ib = body_b_iinv(P, bb);
  const F4 qa = lds_f4(rec + ba), qb = lds_f4(rec + bb);
  const float vs1x = __builtin_fmaf(-c.r1.y, qa.z, qa.x), vs1y = __builtin_fmaf(c.r1.x, qa.z, qa.y);
  const float vs2x = __builtin_fmaf(-c.r2.y, qb.z, qb.x), vs2y = __builtin_fmaf(c.r2.x, qb.z, qb.y);
  const float vrx = vs2x - vs1x, vry = vs2y - vs1y;
  const float vn = vrx * c.n.x + vry * c.n.y;
  const float j1 = (c.K - vn) * c.nMass;
  const float old = c.acc;
  c.acc = fmaxr(old + j1, 0.0f);
  const float vrt = vrx * (-c.n.y) + vry * c.n.x;
  const float jtMax = c.u * c.acc;
  const float jt = -vrt * c.tMass;
  const float jtOld = c.jt;
  c.jt = fclamp_sym(jtOld + jt, jtMax);
  const float d = c.acc - old, e = c.jt - jtOld;
  const float Jx = __builtin_fmaf(c.n.x, d, -(c.n.y * e)), Jy = __builtin_fmaf(c.n.x, e, c.n.y * d);
  float* da = (float*)(rec + ba);
  da[0] = __builtin_fmaf(-Jx, ma, qa.x); da[1] = __builtin_fmaf(-Jy, ma, qa.y);
  da[2] = __builtin_fmaf(ia, c.r1.x * (-Jy) - c.r1.y * (-Jx), qa.z);
  float* db = (float*)(rec + bb);
  db[0] = __builtin_fmaf(Jx, mb, qb.x); db[1] = __builtin_fmaf(Jy, mb, qb.y);
  db[2] = __builtin_fmaf(ib, c.r2.x * Jy - c.r2.y * Jx, qb.z);
}
template <int MODE>
__global__ __launch_bounds__(64) void kb(long long* cyc, float* out, int reps) {
  __shared__ GEnv Es[8];
  const int lane = threadIdx.x, g = lane / 8, s = lane % 8;
  GEnv& E = Es[g];
  if (s < 6) {
    E.vw[s] = make_float4(s == 5 ? 0.f : 0.1f * s + g, s == 5 ? 0.f : 0.2f, s == 5 ? 0.f : 0.01f, 0.f);
    E.bw[s] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  Params P = default_params();
  const int pairs[8][2] = {{0, 1}, {1, 2}, {2, 3}, {4, 0}, {5, 1}, {5, 2}, {4, 5}, {0, 3}};
  HSlot reg[KREG];
  const bool bias = s == 1;
  static_for<0, KREG>([&](auto kc) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    reg[k].r1 = v2(3.f + k, -2.f); reg[k].r2 = v2(-1.f, 4.f - k); reg[k].n = v2(0.6f, 0.8f);
    reg[k].u = 0.5f; reg[k].nMass = 0.3f; reg[k].tMass = 0.2f; reg[k].K = bias ? 0.1f : -0.05f;
    reg[k].acc = 0.f; reg[k].jt = 0.f;
    reg[k].m = (uint32_t)pairs[(k + g) & 7][0] | ((uint32_t)pairs[(k + g) & 7][1] << 3);
  });
  const int nc = 8;
  float4* const rec = bias ? E.bw : E.vw;
  long long t0 = clock64();
  if (s < 2) {
    for (int rep = 0; rep < reps; ++rep) {
#pragma unroll 1
      for (int it = 0; it < 10; ++it) {
        static_for<0, KREG>([&](auto kc) __attribute__((always_inline)) {
          constexpr int k = decltype(kc)::value;
          if (k < nc) { if (MODE == 0) solve_h(P, reg[k], rec); else solve_hs(P, reg[k], rec); }
        });
      }
    }
  }
  long long t1 = clock64();
  float acc = 0.f;
  static_for<0, KREG>([&](auto kc) __attribute__((always_inline)) { acc += reg[decltype(kc)::value].acc + reg[decltype(kc)::value].jt; });
  out[lane] = acc + E.vw[0].x;
  if (lane == 0) cyc[0] = t1 - t0;
}
int main() {
  long long* cyc; float* out; hipMalloc(&cyc, 64); hipMalloc(&out, 1024);
  int reps = 100;
  float h0[64], h1[64];
  for (int r = 0; r < 2; ++r) {
    long long h;
    kb<0><<<1, 64>>>(cyc, out, reps); hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost); hipMemcpy(h0, out, 256, hipMemcpyDeviceToHost);
    printf("solve_h (packed pairs, med3 clamp): %.1f cycles/solve\n", (double)h / reps / 80);
    kb<1><<<1, 64>>>(cyc, out, reps); hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost); hipMemcpy(h1, out, 256, hipMemcpyDeviceToHost);
    printf("scalar restatement: %.1f cycles/solve (results %s)\n", (double)h / reps / 80, memcmp(h0, h1, 256) ? "DIFFER" : "equal");
  }
  return 0;
}
