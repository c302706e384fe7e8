/*
 * amgd_hostmath.h -- the host-side scalar pieces of the smoother setup, shared by the
 * one-GPU driver (amgd_setup.c) and the partitioned driver (amgd_psetup.c): the
 * tridiagonal eigen-solve of Lanczos (tdeig / sec_root, reference amg_setup.c:2616-2735)
 * and the Chebyshev degree (chebsim, amg_setup.c:2412).  Plain C compiled with
 * -ffp-contract=off: every operation rounds as in the reference's ISO-C build.
 */
#ifndef AMGD_HOSTMATH_H
#define AMGD_HOSTMATH_H
#include <float.h>
#include <math.h>

#define EPS (128 * DBL_EPSILON)
static double sum_3(double a, double b, double c) {
  if ((a >= 0 && b >= 0) || (a <= 0 && b <= 0)) return (a + b) + c;
  if ((a >= 0 && c >= 0) || (a <= 0 && c <= 0)) return (a + c) + b;
  return a + (b + c);
}
static double rat_root(double a, double b, double c, double sign) {
  double bh = (fabs(b) + sqrt(b * b + 4 * a * c)) / 2;
  return sign * (b * sign <= 0 ? bh / a : c / bh);
}
/* secular-equation root in [d[ri], d[ri+1]] (amg_setup.c:2638) */
static double sec_root(double *y, const double *d, const double *v, int ri, int n) {
  double dl = d[ri], dr = d[ri + 1], L = dr - dl, x0l = L / 2, x0r = -L / 2;
  double tol = L;
  if (fabs(dl) > tol) tol = fabs(dl);
  if (fabs(dr) > tol) tol = fabs(dr);
  tol *= EPS;
  for (;;) {
    double al = 0, ar = 0, cl = 0, cr = 0, bln = 0, blp = 0, brn = 0, brp = 0, fn = 0, fp = 0;
    double lambda0, lambda;
    if (fabs(x0l) == 0 || x0l < 0) { *y = 0; return dl; }
    if (fabs(x0r) == 0 || x0r > 0) { *y = 0; return dr; }
    lambda0 = fabs(x0l) < fabs(x0r) ? dl + x0l : dr + x0r;
    for (int i = 1; i <= ri; ++i) {
      double den = (d[i] - dl) - x0l, fac = v[i] / den, num = sum_3(d[i], -dr, -2 * x0r);
      fn += v[i] * fac; fac *= fac; ar += fac;
      if (num > 0) brp += fac * num; else brn += fac * num;
      bln += fac * (d[i] - dl);
      cl += fac * x0l * x0l;
    }
    for (int i = ri + 1; i <= n; ++i) {
      double den = (d[i] - dr) - x0r, fac = v[i] / den, num = sum_3(d[i], -dl, -2 * x0l);
      fp += v[i] * fac; fac *= fac; al += fac;
      if (num > 0) blp += fac * num; else bln += fac * num;
      brp += fac * (d[i] - dr);
      cr += fac * x0r * x0r;
    }
    if (lambda0 > 0) fp += lambda0; else fn += lambda0;
    if (v[0] < 0) fp -= v[0], blp -= v[0], brp -= v[0];
    else fn -= v[0], bln -= v[0], brn -= v[0];
    if (fp + fn > 0) {
      x0l = rat_root(1 + al, sum_3(dl, blp, bln), cl, 1);
      lambda = dl + x0l; x0r = x0l - L;
    } else {
      x0r = rat_root(1 + ar, sum_3(dr, brp, brn), cr, -1);
      lambda = dr + x0r; x0l = x0r + L;
    }
    if (fabs(lambda - lambda0) < tol) {
      double ty = 0, fac;
      for (int i = 1; i <= ri; ++i) fac = v[i] / ((d[i] - dl) - x0l), ty += fac * fac;
      for (int i = ri + 1; i <= n; ++i) fac = v[i] / ((d[i] - dr) - x0r), ty += fac * fac;
      *y = 1 / sqrt(1 + ty);
      return lambda;
    }
  }
}
static void tdeig(double *lambda, double *y, double *d, const double *v, int n) {
  double v1 = 0, mn = v[0], mx = v[0];
  for (int i = 1; i <= n; ++i) {
    double vi = fabs(v[i]), a = d[i] - vi, b = d[i] + vi;
    v1 += vi;
    if (a < mn) mn = a;
    if (b > mx) mx = b;
  }
  d[0] = v[0] - v1 < mn ? v[0] - v1 : mn;
  d[n + 1] = v[0] + v1 > mx ? v[0] + v1 : mx;
  for (int i = 0; i <= n; ++i) lambda[i] = sec_root(&y[i], d, v, i, n);
}

static void chebsim(double *m, double *c, double rho, double tol) {   /* amg_setup.c:2412 */
  double alpha = 0.25 * rho * rho, cp = 1, gamma = 1, d, cn;
  *m = 1; *c = rho;
  while (*c > tol) {
    *m += 1;
    d = alpha * (1 + gamma);
    gamma = d / (1 - d);
    cn = (1 + gamma) * rho * (*c) - gamma * cp;
    cp = *c; *c = cn;
  }
}

#endif
