// valu_rates.hip -- issue cost of the instruction kinds the Newton site is made of, on this chip.
//
// Each kernel runs 8 independent dependency chains per lane (so latency is hidden inside one wave too), 8 waves per
// SIMD, and the same chain body kLoop times:
//   mul_add   x = x * a + b as two instructions (v_mul_f32, v_add_f32: the reference's arithmetic, no contraction)
//   div_rn    x = a / x, the correctly rounded binary32 division (v_div_scale x2, v_rcp, fma chain, v_div_fmas,
//             v_div_fixup: the sequence every unproven division site of the Newton site runs)
//   div_plain x = a * rcp(x) refined by the unscaled fma chain (div_unscaled in patch_math.hpp)
//   sqrt_rn   x = sqrt(x + a), correctly rounded (v_sqrt plus the neighbour tests)
//   rcp       x = v_rcp_f32(x + a)
//   pk_mul_add the mul_add chains two at a time as float2 (v_pk_mul_f32, v_pk_add_f32: same per-element rounding)
//   mul_add16 mul_add with 16 chains per lane instead of 8
//   mul_add_v mul_add with a and b in VGPRs (lane-dependent) instead of SGPRs
//   fma       x = fma(x, a, b): one instruction per step (contracted; not the parity arithmetic)
//   add_only  x = x + b
//   mix25     four instructions per step, one of them reading an SGPR operand: ((x * av + bv) * av) + b
//   pk_v      pk_mul_add with a and b in VGPRs
// The program prints, per kernel, the launch time (best of 5, HIP events) and the chain steps per second; VALU
// instructions per step come from the device assembly or a `rocprofv3 --pmc SQ_INSTS_VALU` pass.
//
// usage: valu_rates [loop]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

constexpr int kChains = 8;
typedef float f2 __attribute__((ext_vector_type(2)));

template <int kKind>
__device__ __forceinline__ float step(float x, float a, float b) {
  if constexpr (kKind == 0) {
    return x * a + b;
  } else if constexpr (kKind == 1) {
    return a / x;
  } else if constexpr (kKind == 2) {
    const float y0 = __builtin_amdgcn_rcpf(x);
    const float y = __builtin_fmaf(__builtin_fmaf(-x, y0, 1.0f), y0, y0);
    float q = a * y;
    float r = __builtin_fmaf(-x, q, a);
    q = __builtin_fmaf(r, y, q);
    r = __builtin_fmaf(-x, q, a);
    return __builtin_fmaf(r, y, q);
  } else if constexpr (kKind == 3) {
    return __builtin_sqrtf(x + a);
  } else if constexpr (kKind == 4) {
    return __builtin_amdgcn_rcpf(x + a);
  } else if constexpr (kKind == 8) {
    return __builtin_fmaf(x, a, b);
  } else {
    return x + b;
  }
}

template <int kKind>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_rate(float a, float b, int loop,
                                                                                       float *__restrict__ out) {
  float s = 0.0f;
  if constexpr (kKind == 5 || kKind == 11) {  // packed: kChains scalar chains as kChains / 2 float2 chains
    f2 x[kChains / 2];
    if constexpr (kKind == 11) {  // lane-dependent operands: VGPRs
      a = a + 1e-7f * (float)(threadIdx.x & 7u);
      b = b + 1e-7f * (float)(threadIdx.x & 3u);
    }
    const f2 a2 = {a, a}, b2 = {b, b};
#pragma unroll
    for (int c = 0; c < kChains / 2; ++c) x[c] = f2{1.0f + 0.001f * (float)(threadIdx.x + 7 * c), 1.0f + 0.002f * (float)c};
    for (int k = 0; k < loop; ++k) {
#pragma unroll
      for (int c = 0; c < kChains / 2; ++c) x[c] = x[c] * a2 + b2;
    }
#pragma unroll
    for (int c = 0; c < kChains / 2; ++c) s += x[c].x + x[c].y;
  } else {
    constexpr int kN = kKind == 6 ? 2 * kChains : kChains;
    if constexpr (kKind == 7) {  // lane-dependent operands: VGPRs
      a = a + 1e-7f * (float)(threadIdx.x & 7u);
      b = b + 1e-7f * (float)(threadIdx.x & 3u);
    }
    const float av = 0.9995f + 1e-7f * (float)(threadIdx.x & 7u), bv = 0.0005f + 1e-7f * (float)(threadIdx.x & 3u);
    float x[kN];
#pragma unroll
    for (int c = 0; c < kN; ++c) x[c] = 1.0f + 0.001f * (float)(threadIdx.x + 7 * c);
    for (int k = 0; k < loop; ++k) {
#pragma unroll
      for (int c = 0; c < kN; ++c) {
        if constexpr (kKind == 10) x[c] = ((x[c] * av + bv) * av) + b;
        else x[c] = step<(kKind == 6 || kKind == 7) ? 0 : kKind>(x[c], a, b);
      }
    }
#pragma unroll
    for (int c = 0; c < kN; ++c) s += x[c];
  }
  out[blockIdx.x * 256u + threadIdx.x] = s;
}

template <int kKind>
void run(const char *name, int cus, int loop, float *out, hipEvent_t e0, hipEvent_t e1, int W = 8) {
  const dim3 grid(cus * W), block(256);
  // a, b keep every chain finite and normal: x * 0.999 + 0.001 -> 1; 1.0001 / x oscillates near 1; sqrt(x + 0.5)
  const float a = (kKind == 0 || kKind >= 5) ? (kKind == 10 ? 0.5f : 0.999f) : (kKind == 3 ? 0.5f : (kKind == 4 ? 0.25f : 1.0001f)), b = 0.001f;
  hipLaunchKernelGGL(k_rate<kKind>, grid, block, 0, 0, a, b, loop, out);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_rate<kKind>, grid, block, 0, 0, a, b, loop, out);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.0f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  CHECK(hipGetLastError());
  const double waves = (double)cus * W * 4.0, steps = waves * loop * (kKind == 6 ? 2 : 1) * kChains;  // wave-steps
  // wave64 steps per SIMD per cycle at 2.4 GHz: 1 / (cycles per wave-step)
  const double cyc = (best * 1e-3) * 2.4e9 * (cus * 4.0) / steps;
  std::printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"wave_steps\": %.0f, "
              "\"simd_cycles_per_wave_step_2p4GHz\": %.3f}\n", name, W, best, steps, cyc);
  std::fflush(stdout);
}

int main(int argc, char **argv) {
  const int loop = argc > 1 ? std::atoi(argv[1]) : 2048;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  float *out = nullptr;
  CHECK(hipMalloc(&out, (size_t)cus * 8u * 256u * sizeof(float)));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  run<0>("mul_add", cus, loop, out, e0, e1);
  run<1>("div_rn", cus, loop, out, e0, e1);
  run<2>("div_plain", cus, loop, out, e0, e1);
  run<3>("sqrt_rn", cus, loop, out, e0, e1);
  run<4>("rcp", cus, loop, out, e0, e1);
  run<5>("pk_mul_add", cus, loop, out, e0, e1);
  run<6>("mul_add16", cus, loop, out, e0, e1);
  run<7>("mul_add_v", cus, loop, out, e0, e1);
  run<8>("fma", cus, loop, out, e0, e1);
  run<9>("add_only", cus, loop, out, e0, e1);
  run<10>("mix25", cus, loop, out, e0, e1);
  run<11>("pk_v", cus, loop, out, e0, e1);
  run<0>("mul_add", cus, loop, out, e0, e1, 1);
  run<0>("mul_add", cus, loop, out, e0, e1, 2);
  run<0>("mul_add", cus, loop, out, e0, e1, 4);
  run<5>("pk_mul_add", cus, loop, out, e0, e1, 1);
  CHECK(hipFree(out));
  return 0;
}
