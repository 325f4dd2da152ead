// f64_chain_floor.hip -- the ISA-level floor of a one-lane dependent chain on
// gfx950 (the State chain of sine_test.cpp).
//
// sine_test.cpp's State update per sample (build/sine_test.cpp:55-66):
//     theta += lfo_step; if (theta > two_pi) theta -= two_pi;
// compiles to v_add_f64 -> (v_add_f64, v_cmp_lt_f64) -> s_nop 1 -> two
// v_cndmask_b32 per sample (the module's dspb_seg_chain_c2b512).  This tool
// times that chain on one lane with the shader clock (s_memtime) against the
// 100 MHz real-time clock, and the chains it is made of, so that the floor is
// measured rather than asserted.  Not part of the product.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o /tmp/f64_floor tools/diag/f64_chain_floor.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr double kTwoPi = 6.28318530717958647692;

template <int kKind>
__global__ void chain(double step, float stepf, long long n, double *out, long long *cyc, long long *rt) {
    if (threadIdx.x != 0) return;
    double ph = 0.0;
    float y = 0.f, z = 0.3f;
    const long long t0 = clock64(), r0 = wall_clock64();
    for (long long i = 0; i < n; i += 32) {
#pragma unroll
      for (int u = 0; u < 32; ++u) {  // (unrolled: the loop's own branch off the chain)
        if constexpr (kKind == 0) {  // sine_test's phase update
            ph += step;
            if (ph > kTwoPi) ph -= kTwoPi;
        } else if constexpr (kKind == 1) {  // dependent f64 adds
            ph += step;
        } else if constexpr (kKind == 2) {  // dependent f32 adds
            y += stepf;
        } else if constexpr (kKind == 3) {  // dependent f32 multiply then add (a one-pole's chain)
            y = y * stepf + z;
        } else {  // the phase update as a select of the subtrahend (same bits: t - 0 == t)
            const double t = ph + step;
            ph = t - (t > kTwoPi ? kTwoPi : 0.0);
        }
      }
    }
    const long long t1 = clock64(), r1 = wall_clock64();
    out[0] = ph + (double)y;
    cyc[0] = t1 - t0;
    rt[0] = r1 - r0;
}

template <int K>
static void run(const char *name, long long n, int per_iter_ops) {
    double *out;
    long long *cyc, *rt;
    hipMalloc(&out, 8);
    hipMalloc(&cyc, 8);
    hipMalloc(&rt, 8);
    for (int rep = 0; rep < 2; ++rep) {  // the first launch warms the clock
        hipLaunchKernelGGL(chain<K>, dim3(1), dim3(64), 0, 0, 0.0523598775598298873, 0.999f, n, out, cyc, rt);
        hipDeviceSynchronize();
    }
    long long c = 0, r = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&r, rt, 8, hipMemcpyDeviceToHost);
    const double ns = (double)r * 10.0 / (double)n;  // wall_clock64: 100 MHz
    const double cpi = (double)c / (double)n;
    std::printf("{\"chain\": \"%s\", \"iterations\": %lld, \"shader_cycles_per_iter\": %.3f, "
                "\"ns_per_iter\": %.4f, \"sclk_ghz\": %.3f, \"ops_per_iter\": %d}\n",
                name, n, cpi, ns, cpi / ns, per_iter_ops);
    hipFree(out);
    hipFree(cyc);
    hipFree(rt);
}

int main() {
    const long long n = 1 << 24;
    run<0>("sine_test phase update (v_add_f64 -> v_add_f64 + v_cmp_lt_f64 -> v_cndmask x2)", n, 5);
    run<4>("phase update as t - (t > 2pi ? 2pi : 0)", n, 5);
    run<1>("dependent v_add_f64", n, 1);
    run<2>("dependent v_add_f32", n, 1);
    run<3>("dependent v_mul_f32 -> v_add_f32", n, 2);
    return 0;
}
