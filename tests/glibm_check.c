// glibm_check.c -- checks csrc/rrt_glibm.h bit for bit against the host C library (test harness).
//
// Built and run by tests/test_glibm.py:
//   gcc -O2 -mfma -ffp-contract=off -fopenmp -I<csrc> glibm_check.c -lm
// -ffp-contract=off keeps every product and sum separately rounded except the explicit fma()
// calls, which -mfma turns into the same vfmadd instructions glibc's FMA build uses.
//
// Modes (one line of JSON each):
//   sampler K0 K1   every Xi = k / RAND_MAX for k in [K0, K1) -- all the values random_uniform()
//                   can return (random_util.h:11-14) -- through the reference's call sites:
//                   cos/sin(2 PI Xi) (sampler.cpp:53-55), acos(Xi) and sinf/cosf of
//                   (float)acos(Xi), (float)(2 PI Xi) (sampler.cpp:20-25)
//   floats F0 F1    sinf and cosf on every float whose bit pattern is in [F0, F1)
//   random N SEED   N random arguments for each of sin, cos (|x| < 105414350), acos (whole line),
//                   sinf, cosf (|x| < 120), half uniform in value, half log-uniform in magnitude,
//                   and atan2 on random pairs and on the environment lookup's unit directions
//   specials        zeros, infinities, NaNs, +-1 and the branch boundaries of every function
//   mf K0 K1        the microfacet sampler (bsdf.cpp:76-86) on every Xi = k / RAND_MAX, k in
//                   [K0, K1): log(1 - Xi), then for three roughnesses atan(sqrt(-a^2 log(1 - Xi))),
//                   tan of that angle and exp(-tan^2 / a^2), each on the library's own inputs
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rrt_glibm.h"

#define PI_REF 3.14159265358979323  // misc.h:11

// the library's functions, called through volatile pointers so the compiler cannot fold them
static double (*volatile lib_sin)(double) = sin;
static double (*volatile lib_cos)(double) = cos;
static double (*volatile lib_acos)(double) = acos;
static float (*volatile lib_sinf)(float) = sinf;
static float (*volatile lib_cosf)(float) = cosf;
static double (*volatile lib_atan2)(double, double) = atan2;
static double (*volatile lib_exp)(double) = exp;
static double (*volatile lib_log)(double) = log;
static double (*volatile lib_erf)(double) = erf;
static double (*volatile lib_atan)(double) = atan;
static double (*volatile lib_tan)(double) = tan;

static int same_d(double a, double b) { uint64_t x, y; memcpy(&x, &a, 8); memcpy(&y, &b, 8); return x == y || (a != a && b != b); }
static int same_f(float a, float b) { uint32_t x, y; memcpy(&x, &a, 4); memcpy(&y, &b, 4); return x == y || (a != a && b != b); }

enum { F_SIN, F_COS, F_ACOS, F_ACOSF, F_SINF, F_COSF, F_SINF_T, F_COSF_T, F_ATAN2, F_EXP, F_LOG, F_ERF, F_ATAN, F_TAN, NF };
static const char* names[NF] = {"sin", "cos", "acos", "acos_to_float", "sinf", "cosf", "sinf_theta", "cosf_theta", "atan2",
                                "exp", "log", "erf", "atan", "tan"};
static long long bad[NF], tested[NF];
static double first_bad[NF];

static void note(int f, int ok, double arg) {
  if (!ok) {
#pragma omp critical
    {
      if (bad[f] == 0) first_bad[f] = arg;
      bad[f]++;
    }
  }
}

static void report(const char* mode) {
  printf("{\"mode\": \"%s\"", mode);
  for (int f = 0; f < NF; ++f)
    if (tested[f]) printf(", \"%s\": [%lld, %lld, %.17g]", names[f], tested[f], bad[f], first_bad[f]);
  printf("}\n");
}

static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// a random double: value-uniform in [-lim, lim] or magnitude log-uniform below lim
static double rand_arg(uint64_t* s, double lim) {
  const uint64_t r = splitmix(s);
  if (r & 1) return ((double)(splitmix(s) >> 11) * 0x1p-53 * 2 - 1) * lim;
  double v;
  do {
    uint64_t b = splitmix(s) & 0x7fffffffffffffffull;
    memcpy(&v, &b, 8);
  } while (!(v < lim));
  return (r & 2) ? -v : v;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  if (!strcmp(argv[1], "sampler") && argc == 4) {
    const long long k0 = atoll(argv[2]), k1 = atoll(argv[3]);
#pragma omp parallel for schedule(static, 65536) reduction(+ : tested[:NF])
    for (long long k = k0; k < k1; ++k) {
      const double xi = ((double)(int)k) / 2147483647.0;   // random_util.h: rand() / RAND_MAX
      const double th = 2. * PI_REF * xi;                   // sampler.cpp:53 and :21
      note(F_SIN, same_d(rrt_glibm_sin(th), lib_sin(th)), th);
      note(F_COS, same_d(rrt_glibm_cos(th), lib_cos(th)), th);
      const double a = rrt_glibm_acos(xi), b = lib_acos(xi);
      note(F_ACOS, same_d(a, b), xi);
      note(F_ACOSF, same_f((float)a, (float)b), xi);
      const float ft = (float)b, fp = (float)th;
      note(F_SINF_T, same_f(rrt_glibm_sinf(ft), lib_sinf(ft)), ft);
      note(F_COSF_T, same_f(rrt_glibm_cosf(ft), lib_cosf(ft)), ft);
      note(F_SINF, same_f(rrt_glibm_sinf(fp), lib_sinf(fp)), fp);
      note(F_COSF, same_f(rrt_glibm_cosf(fp), lib_cosf(fp)), fp);
      tested[F_SIN]++; tested[F_COS]++; tested[F_ACOS]++; tested[F_ACOSF]++;
      tested[F_SINF_T]++; tested[F_COSF_T]++; tested[F_SINF]++; tested[F_COSF]++;
    }
    report("sampler");
  } else if (!strcmp(argv[1], "floats") && argc == 4) {
    const long long f0 = atoll(argv[2]), f1 = atoll(argv[3]);
#pragma omp parallel for schedule(static, 65536) reduction(+ : tested[:NF])
    for (long long b = f0; b < f1; ++b) {
      const uint32_t u = (uint32_t)b;
      float x;
      memcpy(&x, &u, 4);
      note(F_SINF, same_f(rrt_glibm_sinf(x), lib_sinf(x)), x);
      note(F_COSF, same_f(rrt_glibm_cosf(x), lib_cosf(x)), x);
      tested[F_SINF]++; tested[F_COSF]++;
    }
    report("floats");
  } else if (!strcmp(argv[1], "random") && argc == 4) {
    const long long n = atoll(argv[2]);
    const uint64_t seed = strtoull(argv[3], 0, 10);
#pragma omp parallel reduction(+ : tested[:NF])
    {
      int nt = 1, id = 0;
#ifdef _OPENMP
      extern int omp_get_num_threads(void), omp_get_thread_num(void);
      nt = omp_get_num_threads(); id = omp_get_thread_num();
#endif
      uint64_t s = seed * 0x100000001B3ull + (uint64_t)id * 0x9E3779B97F4A7C15ull;
      for (long long i = id; i < n; i += nt) {
        const double x = rand_arg(&s, 105414350.0);
        note(F_SIN, same_d(rrt_glibm_sin(x), lib_sin(x)), x);
        note(F_COS, same_d(rrt_glibm_cos(x), lib_cos(x)), x);
        const double c = (splitmix(&s) & 7) == 0 ? rand_arg(&s, 2.0) : rand_arg(&s, 1.0);
        note(F_ACOS, same_d(rrt_glibm_acos(c), lib_acos(c)), c);
        const float f = (float)rand_arg(&s, 120.0);
        note(F_SINF, same_f(rrt_glibm_sinf(f), lib_sinf(f)), f);
        note(F_COSF, same_f(rrt_glibm_cosf(f), lib_cosf(f)), f);
        // atan2: a random pair (each coordinate value- or log-uniform, either sign), or the
        // environment light's miss lookup atan2(-u.z, u.x) of a random unit direction
        double ya, xa;
        if (splitmix(&s) & 1) {
          ya = rand_arg(&s, (splitmix(&s) & 1) ? 1e300 : 2.0);
          xa = rand_arg(&s, (splitmix(&s) & 1) ? 1e300 : 2.0);
        } else {
          const double dx = rand_arg(&s, 1.0), dy = rand_arg(&s, 1.0), dz = rand_arg(&s, 1.0);
          const double r = 1.0 / sqrt(dx * dx + dy * dy + dz * dz);   // Vector3D::unit
          ya = -(dz * r);
          xa = dx * r;
          note(F_ACOS, same_d(rrt_glibm_acos(dy * r), lib_acos(dy * r)), dy * r);
        }
        note(F_ATAN2, same_d(rrt_glibm_atan2(ya, xa), lib_atan2(ya, xa)), ya);
        // the microfacet functions: exp over its whole finite range and the subnormal results,
        // log of any positive (subnormals included, sometimes near 1 or negative), erf, atan on
        // the whole line, tan on the restated domain |x| <= 25
        const double e = (splitmix(&s) & 1) ? rand_arg(&s, 760.0) : rand_arg(&s, 1.0);
        note(F_EXP, same_d(rrt_glibm_exp(e), lib_exp(e)), e);
        const uint64_t lr = splitmix(&s);
        const double l = (lr & 3) == 0 ? 1.0 + rand_arg(&s, 0.1) : (lr & 31) == 1 ? -rand_arg(&s, 1e300) : fabs(rand_arg(&s, 1e308));
        note(F_LOG, same_d(rrt_glibm_log(l), lib_log(l)), l);
        const double ef = (splitmix(&s) & 1) ? rand_arg(&s, 7.0) : rand_arg(&s, 1e300);
        note(F_ERF, same_d(rrt_glibm_erf(ef), lib_erf(ef)), ef);
        const double at = (splitmix(&s) & 1) ? rand_arg(&s, 20.0) : rand_arg(&s, 1e300);
        note(F_ATAN, same_d(rrt_glibm_atan(at), lib_atan(at)), at);
        const double tn = (splitmix(&s) & 1) ? rand_arg(&s, 3.2) : rand_arg(&s, 25.0);
        note(F_TAN, same_d(rrt_glibm_tan(tn), lib_tan(tn)), tn);
        tested[F_SIN]++; tested[F_COS]++; tested[F_ACOS]++; tested[F_SINF]++; tested[F_COSF]++;
        tested[F_ATAN2]++; tested[F_EXP]++; tested[F_LOG]++; tested[F_ERF]++; tested[F_ATAN]++; tested[F_TAN]++;
      }
    }
    report("random");
  } else if (!strcmp(argv[1], "mf") && argc == 4) {
    const long long k0 = atoll(argv[2]), k1 = atoll(argv[3]);
    static const double alphas[3] = {0.05, 0.25, 0.5};
#pragma omp parallel for schedule(static, 65536) reduction(+ : tested[:NF])
    for (long long k = k0; k < k1; ++k) {
      const double xi = ((double)(int)k) / 2147483647.0;
      const double lg = lib_log(1 - xi);                      // bsdf.cpp:78
      note(F_LOG, same_d(rrt_glibm_log(1 - xi), lg), 1 - xi);
      tested[F_LOG]++;
      for (int a = 0; a < 3; ++a) {
        const double a2 = alphas[a] * alphas[a];
        const double q = sqrt(-a2 * lg);
        const double th = lib_atan(q);                        // theta_h
        note(F_ATAN, same_d(rrt_glibm_atan(q), th), q);
        const double t = lib_tan(th);                         // bsdf.cpp:83
        note(F_TAN, same_d(rrt_glibm_tan(th), t), th);
        const double ea = -t * t / a2;                        // bsdf.cpp:84
        note(F_EXP, same_d(rrt_glibm_exp(ea), lib_exp(ea)), ea);
        tested[F_ATAN]++; tested[F_TAN]++; tested[F_EXP]++;
      }
    }
    report("mf");
  } else if (!strcmp(argv[1], "specials")) {
    // every branch boundary of the restated routines (high words from s_sin.c, e_asin.c,
    // e_atan2.c, s_sinf.c), 64 ulps either side, both signs, plus zeros, infinities, NaNs
    static const uint32_t his[] = {0x3e400000u, 0x3e500000u, 0x3feb6000u, 0x400368fdu, 0x419921fbu,
                                   0x3c880000u, 0x3fc00000u, 0x3fd00000u, 0x3fe00000u, 0x3fe80000u,
                                   0x3fed8000u, 0x3fee8000u, 0x3fef0000u, 0x3ff00000u, 0x7ff00000u,
                                   0x3fb00000u, 0x20b00000u, 0x5f300000u, 0x00100000u, 0x0u};
    double pts[2 * 20 * 129 + 16];
    int np = 0;
    for (unsigned h = 0; h < sizeof(his) / sizeof(his[0]); ++h)
      for (int d = -64; d <= 64; ++d) {
        const uint64_t b = ((uint64_t)his[h] << 32) + (uint64_t)(int64_t)d;
        double v;
        memcpy(&v, &b, 8);
        pts[np++] = v;
        pts[np++] = -v;
      }
    const double extra[] = {0.0, -0.0, INFINITY, -INFINITY, NAN, 1.0, -1.0, 0.126, -0.126, 0.0625,
                            3.14159265358979323, 1.5707963267948966, 2.426265, 105414350.0};
    for (unsigned i = 0; i < sizeof(extra) / sizeof(extra[0]); ++i) pts[np++] = extra[i];
    // the microfacet functions' branch boundaries (e_exp.c, e_log.c, s_erf.c, s_atan.c, s_tan.c)
    static const uint32_t mhis[] = {0x3c900000u, 0x40800000u, 0x40900000u, 0x40862e42u, 0x408633ceu, 0x40874910u,
                                    0x3fee0000u, 0x3ff10900u, 0x3fe60000u, 0x00100000u, 0x000fffffu, 0x3e300000u,
                                    0x3feb0000u, 0x3ff40000u, 0x4006db6eu, 0x40180000u, 0x00800000u, 0x3e4bb67au,
                                    0x3fb00000u, 0x40300000u, 0x43349ff2u, 0x3e4b096cu, 0x3faf212du, 0x3fe92f1au,
                                    0x40390000u, 0x3ff921fbu, 0x400921fbu, 0x4012d97cu};
    double mpts[2 * 28 * 129];
    int nm = 0;
    for (unsigned h = 0; h < sizeof(mhis) / sizeof(mhis[0]); ++h)
      for (int d = -64; d <= 64; ++d) {
        const uint64_t b = ((uint64_t)mhis[h] << 32) + (uint64_t)(int64_t)d;
        double v;
        memcpy(&v, &b, 8);
        mpts[nm++] = v;
        mpts[nm++] = -v;
      }
    for (int i = 0; i < nm + np; ++i) {
      const double x = i < nm ? mpts[i] : pts[i - nm];
      note(F_EXP, same_d(rrt_glibm_exp(x), lib_exp(x)), x);
      note(F_LOG, same_d(rrt_glibm_log(x), lib_log(x)), x);
      note(F_ERF, same_d(rrt_glibm_erf(x), lib_erf(x)), x);
      note(F_ATAN, same_d(rrt_glibm_atan(x), lib_atan(x)), x);
      tested[F_EXP]++; tested[F_LOG]++; tested[F_ERF]++; tested[F_ATAN]++;
      if (fabs(x) <= 25.0 || x != x || isinf(x)) {
        note(F_TAN, same_d(rrt_glibm_tan(x), lib_tan(x)), x);
        tested[F_TAN]++;
      }
    }
    for (int i = 0; i < np; ++i) {
      const double x = pts[i];
      note(F_SIN, same_d(rrt_glibm_sin(x), lib_sin(x)), x);
      note(F_COS, same_d(rrt_glibm_cos(x), lib_cos(x)), x);
      note(F_ACOS, same_d(rrt_glibm_acos(x), lib_acos(x)), x);
      const float f = (float)x;
      if (fabsf(f) < 120.0f) {
        note(F_SINF, same_f(rrt_glibm_sinf(f), lib_sinf(f)), f);
        note(F_COSF, same_f(rrt_glibm_cosf(f), lib_cosf(f)), f);
        tested[F_SINF]++; tested[F_COSF]++;
      }
      tested[F_SIN]++; tested[F_COS]++; tested[F_ACOS]++;
      for (int j = 0; j < np; j += 7) {
        note(F_ATAN2, same_d(rrt_glibm_atan2(x, pts[j]), lib_atan2(x, pts[j])), x);
        note(F_ATAN2, same_d(rrt_glibm_atan2(pts[j], x), lib_atan2(pts[j], x)), pts[j]);
        tested[F_ATAN2] += 2;
      }
    }
    report("specials");
  } else {
    return 2;
  }
  long long total = 0;
  for (int f = 0; f < NF; ++f) total += bad[f];
  return total ? 1 : 0;
}
