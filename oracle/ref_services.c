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
