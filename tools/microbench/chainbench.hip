// Diagnostic (not product): cycles per contact solve of the lane-pair kernel's serial halves, three
// ways of carrying the body records between consecutive solves of one half:
//   0  the product: grp::solve_h<32> (records read from and written to LDS by every solve)
//   1  LDS records, the next contact's two records read BEFORE this contact's writes and replaced by
//      this contact's results where the two contacts share a body (forwarding)
//   2  the half's six body records in registers, the next contact's inputs forwarded the same way
// All three run the same solve_h_core operations on the same values (results compared bit for bit).
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -o chainbench chainbench.hip
#include "../../marl-soccer_amd/csrc/ms_env.hip"
using namespace grp;
hipError_t ms_kstep_launch(int, int, dim3, hipStream_t, const DevState&, const Params&, int, const float*, float*, float*,
                           uint8_t*, uint8_t*, int8_t*, int32_t*, Counters*, int) {
  return hipErrorNotSupported;  // (the K-step unit is not linked into the microbenchmark)
}

constexpr int NC = 6;
struct BL {
  float4 vw[6][32];
  float4 pad[4];
  float4 bw[6][32];
  float2 mass[8];
  float fill[3000];  // 20 KB per workgroup: at most 8 per CU, two waves per SIMD
};

__device__ __forceinline__ V2 sel2(bool c, V2 a, V2 b) { return v2(c ? a.x : b.x, c ? a.y : b.y); }

template <int MODE, int PAT>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) void kb(long long* cyc, float* out,
                                                                                     int reps) {
  __shared__ BL L;
  const int lane = threadIdx.x, p = lane >> 1, s = lane & 1;
  const bool bias = s == 1;
  if (s == 0) {
    for (int b = 0; b < 6; ++b) {
      L.vw[b][p] = make_float4(b == 5 ? 0.f : 0.1f * b + 0.01f * p, b == 5 ? 0.f : 0.2f, b == 5 ? 0.f : 0.01f, 0.f);
      L.bw[b][p] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  if (lane < 8) {
    const Params P = default_params();
    L.mass[lane] = make_float2(body_minv(P, lane), body_iinv(P, lane));
  }
  __syncthreads();
  const Params P = default_params();
  // PAT 0: a pile-up chain (consecutive contacts share a body); 1: alternating disjoint bodies
  const int pairs0[NC][2] = {{0, 1}, {0, 1}, {5, 0}, {5, 0}, {4, 0}, {5, 1}};
  const int pairs1[NC][2] = {{0, 1}, {2, 3}, {5, 0}, {4, 2}, {5, 1}, {5, 3}};
  HSlot reg[NC];
  static_for<0, NC>([&](auto kc) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    reg[k].r1 = v2(3.f + k, -2.f); reg[k].r2 = v2(-1.f, 4.f - k); reg[k].n = v2(0.6f, 0.8f);
    reg[k].u = bias ? 0.f : 0.5f; reg[k].nMass = 0.3f; reg[k].tMass = bias ? 0.f : 0.2f;
    reg[k].K = bias ? 0.1f + 0.01f * p : -0.05f;
    reg[k].acc = 0.f; reg[k].jt = 0.f;
    const int a = PAT ? pairs1[k][0] : pairs0[k][0], b = PAT ? pairs1[k][1] : pairs0[k][1];
    reg[k].m = (uint32_t)a | ((uint32_t)b << 3);
  });
  float4* const rec = bias ? &L.bw[0][p] : &L.vw[0][p];
  float R[6][3];
  if (MODE == 2) {
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const F4 q = lds_f4(rec + b * 32);
      R[b][0] = q.x; R[b][1] = q.y; R[b][2] = q.z;
    }
  }
  __builtin_amdgcn_s_setprio(3);
  long long t0 = clock64();
  if (MODE == 0) {
    for (int rep = 0; rep < reps; ++rep) {
#pragma unroll 1
      for (int it = 0; it < 10; ++it) {
        static_for<0, NC>([&](auto kc) __attribute__((always_inline)) {
          constexpr int k = decltype(kc)::value;
          asm volatile("" : "+v"(reg[k].m));
          solve_h<32>(P, reg[k], rec, L.mass);
        });
      }
    }
  } else if (MODE == 3 || MODE == 4) {
    // solve_h with the read quads held to the end (no write-after-write wait on their 4th register);
    // MODE 4: the two record byte addresses precomputed per slot (one packed word)
    uint32_t ad[NC];
    static_for<0, NC>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      const uint32_t base = (uint32_t)((char*)rec - (char*)&L);
      ad[k] = (base + CS_BA(reg[k].m) * 512u) | ((base + CS_BB(reg[k].m) * 512u) << 16);
    });
    for (int rep = 0; rep < reps; ++rep) {
#pragma unroll 1
      for (int it = 0; it < 10; ++it) {
        static_for<0, NC>([&](auto kc) __attribute__((always_inline)) {
          constexpr int k = decltype(kc)::value;
          asm volatile("" : "+v"(reg[k].m), "+v"(ad[k]));
          HSlot& c = reg[k];
          const int ba = CS_BA(c.m), bb = CS_BB(c.m);
          float4* pa;
          float4* pb;
          if (MODE == 4) {
            pa = (float4*)((char*)&L + (ad[k] & 0xffffu));
            pb = (float4*)((char*)&L + (ad[k] >> 16));
          } else {
            pa = rec + ba * 32;
            pb = rec + bb * 32;
          }
          const F4 qa = lds_f4(pa), qb = lds_f4(pb);
          const float2 A = L.mass[ba], B = L.mass[bb];
          V2 xa, xb;
          float xwa, xwb;
          solve_h_core(c, A.x, A.y, B.x, B.y, v2(qa.x, qa.y), qa.z, v2(qb.x, qb.y), qb.z, xa, xwa, xb, xwb);
          float* da = (float*)pa;
          da[0] = xa.x; da[1] = xa.y; da[2] = xwa;
          float* db = (float*)pb;
          db[0] = xb.x; db[1] = xb.y; db[2] = xwb;
          asm volatile("" ::"v"(qa), "v"(qb));
        });
      }
    }
  } else {
    // the first contact's inputs
    V2 va, vb;
    float wa, wb;
    {
      const int ba = CS_BA(reg[0].m), bb = CS_BB(reg[0].m);
      if (MODE == 1) {
        const F4 qa = lds_f4(rec + ba * 32), qb = lds_f4(rec + bb * 32);
        va = v2(qa.x, qa.y); wa = qa.z; vb = v2(qb.x, qb.y); wb = qb.z;
      } else {
        va = v2(0.f, 0.f); vb = va; wa = 0.f; wb = 0.f;
#pragma unroll
        for (int b = 0; b < 6; ++b) {
          if (ba == b) { va = v2(R[b][0], R[b][1]); wa = R[b][2]; }
          if (bb == b) { vb = v2(R[b][0], R[b][1]); wb = R[b][2]; }
        }
      }
    }
    for (int rep = 0; rep < reps; ++rep) {
#pragma unroll 1
      for (int it = 0; it < 10; ++it) {
        static_for<0, NC>([&](auto kc) __attribute__((always_inline)) {
          constexpr int k = decltype(kc)::value;
          constexpr int kn = k + 1 < NC ? k + 1 : 0;
          asm volatile("" : "+v"(reg[k].m));
          HSlot& c = reg[k];
          const int ba = CS_BA(c.m), bb = CS_BB(c.m);
          const int na_ = CS_BA(reg[kn].m), nb_ = CS_BB(reg[kn].m);
          const float2 A = L.mass[ba], B = L.mass[bb];
          // the next contact's records as they stand before this contact's writes
          V2 pa, pb;
          float pwa, pwb;
          F4 pqa = F4{0.f, 0.f, 0.f, 0.f}, pqb = pqa;
          if (MODE == 1) {
            pqa = lds_f4(rec + na_ * 32);
            pqb = lds_f4(rec + nb_ * 32);
            pa = v2(pqa.x, pqa.y); pwa = pqa.z; pb = v2(pqb.x, pqb.y); pwb = pqb.z;
            __builtin_amdgcn_sched_barrier(0);  // the reads issue before this contact's chain
          } else {
            pa = v2(0.f, 0.f); pb = pa; pwa = 0.f; pwb = 0.f;
#pragma unroll
            for (int b = 0; b < 6; ++b) {
              if (na_ == b) { pa = v2(R[b][0], R[b][1]); pwa = R[b][2]; }
              if (nb_ == b) { pb = v2(R[b][0], R[b][1]); pwb = R[b][2]; }
            }
          }
          V2 xa, xb;
          float xwa, xwb;
          solve_h_core(c, A.x, A.y, B.x, B.y, va, wa, vb, wb, xa, xwa, xb, xwb);
          if (MODE == 1) {
            float* da = (float*)(rec + ba * 32);
            da[0] = xa.x; da[1] = xa.y; da[2] = xwa;
            float* db = (float*)(rec + bb * 32);
            db[0] = xb.x; db[1] = xb.y; db[2] = xwb;
          } else {
#pragma unroll
            for (int b = 0; b < 6; ++b) {
              if (ba == b) { R[b][0] = xa.x; R[b][1] = xa.y; R[b][2] = xwa; }
              if (bb == b) { R[b][0] = xb.x; R[b][1] = xb.y; R[b][2] = xwb; }
            }
          }
          // forward: a record this contact wrote replaces the early read
          va = na_ == ba ? xa : (na_ == bb ? xb : pa);
          wa = na_ == ba ? xwa : (na_ == bb ? xwb : pwa);
          vb = nb_ == ba ? xa : (nb_ == bb ? xb : pb);
          wb = nb_ == ba ? xwa : (nb_ == bb ? xwb : pwb);
          // (MODE 1) the early reads' whole destination quads stay allocated until here: reusing their
          // unused 4th register as a temporary makes the chain wait for the read (write-after-write)
          if (MODE == 1) asm volatile("" ::"v"(pqa), "v"(pqb));
        });
      }
    }
    if (MODE == 2) {
#pragma unroll
      for (int b = 0; b < 6; ++b) {
        float* d = (float*)(rec + b * 32);
        d[0] = R[b][0]; d[1] = R[b][1]; d[2] = R[b][2];
      }
    }
  }
  long long t1 = clock64();
  __builtin_amdgcn_s_setprio(0);
  float acc = 0.f;
  static_for<0, NC>([&](auto kc) __attribute__((always_inline)) {
    acc += reg[decltype(kc)::value].acc + reg[decltype(kc)::value].jt;
  });
  __syncthreads();
  float v = 0.f;
  for (int b = 0; b < 6; ++b) v += L.vw[b][p].x + L.vw[b][p].y + L.vw[b][p].z + L.bw[b][p].x + L.bw[b][p].z;
  out[blockIdx.x * 64 + lane] = acc + v;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE, int PAT>
double run(long long* cyc, float* out, int grid, int reps, float* host) {
  kb<MODE, PAT><<<grid, 64>>>(cyc, out, reps);
  hipDeviceSynchronize();
  std::vector<long long> h(grid);
  hipMemcpy(h.data(), cyc, 8 * grid, hipMemcpyDeviceToHost);
  hipMemcpy(host, out, 4 * 64 * grid, hipMemcpyDeviceToHost);
  double s = 0;
  for (auto x : h) s += (double)x;
  return s / grid / reps / (10.0 * NC);
}

int main() {
  const int GMAX = 2048, reps = 50;
  long long* cyc;
  float* out;
  hipMalloc(&cyc, 8 * GMAX);
  hipMalloc(&out, 4 * 64 * GMAX);
  std::vector<float> h0(64 * GMAX), h1(64 * GMAX), h2(64 * GMAX);
  for (int grid : {1, 2048}) {
    for (int r = 0; r < 2; ++r) {
      {
        double c3 = run<3, 0>(cyc, out, grid, reps, h1.data());
        double c4 = run<4, 0>(cyc, out, grid, reps, h2.data());
        double c0 = run<0, 0>(cyc, out, grid, reps, h0.data());
        const bool e3 = memcmp(h0.data(), h1.data(), 4 * 64 * grid) == 0, e4 = memcmp(h0.data(), h2.data(), 4 * 64 * grid) == 0;
        printf("grid %4d pile-up chain: product %.1f, quads held %.1f (%s), + precomputed addresses %.1f (%s)\n", grid, c0,
               c3, e3 ? "equal" : "DIFFER", c4, e4 ? "equal" : "DIFFER");
      }
      double c0 = run<0, 0>(cyc, out, grid, reps, h0.data());
      double c1 = run<1, 0>(cyc, out, grid, reps, h1.data());
      double c2 = run<2, 0>(cyc, out, grid, reps, h2.data());
      const bool e1 = memcmp(h0.data(), h1.data(), 4 * 64 * grid) == 0, e2 = memcmp(h0.data(), h2.data(), 4 * 64 * grid) == 0;
      printf("grid %4d pile-up chain: product %.1f, LDS+forward %.1f (%s), registers %.1f (%s) cycles/solve\n", grid, c0,
             c1, e1 ? "equal" : "DIFFER", c2, e2 ? "equal" : "DIFFER");
      c0 = run<0, 1>(cyc, out, grid, reps, h0.data());
      c1 = run<1, 1>(cyc, out, grid, reps, h1.data());
      c2 = run<2, 1>(cyc, out, grid, reps, h2.data());
      const bool f1 = memcmp(h0.data(), h1.data(), 4 * 64 * grid) == 0, f2 = memcmp(h0.data(), h2.data(), 4 * 64 * grid) == 0;
      printf("grid %4d disjoint pairs: product %.1f, LDS+forward %.1f (%s), registers %.1f (%s) cycles/solve\n", grid, c0,
             c1, f1 ? "equal" : "DIFFER", c2, f2 ? "equal" : "DIFFER");
    }
  }
  return 0;
}
