/* ref_services.c -- TEST INFRASTRUCTURE ONLY.
 *
 * The few plugin_header.h host services the stock reference plugins built
 * into oracle/_ref need at load time (ref build/plugin_header.h:33-72;
 * registered by name in ref compiler.cpp:311-386).  Plain libm, IEEE.
 */
#include <math.h>
#include <stdlib.h>

double sin_64(double d) { return sin(d); }
double cos_64(double d) { return cos(d); }
double tan_64(double d) { return tan(d); }
double sqrt_64(double d) { return sqrt(d); }
double exp_64(double d) { return exp(d); }
double pow_64(double a, double b) { return pow(a, b); }
double fabs_64(double d) { return fabs(d); }
float sin_32(float d) { return sinf(d); }
float cos_32(float d) { return cosf(d); }
float fabs_32(float d) { return fabsf(d); }
float sqrt_32(float d) { return sqrtf(d); }

/* Simple bump allocator on malloc: initialization_context is ignored. */
float *allocate_buffer(int n, void *ctx) { (void)ctx; return (float *)calloc((size_t)n, sizeof(float)); }
void *allocate_bytes(int n, void *ctx) { (void)ctx; return calloc((size_t)n, 1); }
float **allocate_buffers(int n, int c, void *ctx)
{
    float **p = (float **)calloc((size_t)c, sizeof(float *));
    for (int i = 0; i < c; ++i) p[i] = allocate_buffer(n, ctx);
    return p;
}

/* Array and spectral services used by build/buffer_test.cpp at load time.
 * fft_forward / fft_reverse restate IPP's CToC transforms with
 * IPP_FFT_DIV_BY_SQRTN (ref dsp.cpp:74-132) as a float64 DFT. */
void set_array(float v, float *out, int n) { for (int i = 0; i < n; ++i) out[i] = v; }
void gain_32_array(float *in, float *out, float g, int n) { for (int i = 0; i < n; ++i) out[i] = in[i] * g; }
void *fft_initialize(void *ctx) { return ctx; }
static void dft64(const float *re, const float *im, float *ore, float *oim, int n, int sign)
{
    const double tp = 6.283185307179586476925286766559;
    for (int k = 0; k < n; ++k) {
        double sr = 0.0, si = 0.0;
        for (int t = 0; t < n; ++t) {
            const double a = sign * tp * (double)((long long)k * t % n) / n;
            const double xr = re[t], xi = im ? im[t] : 0.0;
            sr += xr * cos(a) - xi * sin(a);
            si += xr * sin(a) + xi * cos(a);
        }
        ore[k] = (float)(sr / sqrt((double)n));
        if (oim) oim[k] = (float)(si / sqrt((double)n));
    }
}
void fft_forward(float *in, float *re, float *im, int n, void *ctx) { (void)ctx; dft64(in, 0, re, im, n, -1); }
void fft_reverse(float *re, float *im, float *out, int n, void *ctx) { (void)ctx; dft64(re, im, out, 0, n, +1); }
