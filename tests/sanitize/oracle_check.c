/* oracle_check.c -- host sanitizer driver (ASan/UBSan on host code) for the oracle
 * (oracle/pb_oracle.c, test infrastructure). Runs every restated routine on small, odd shapes
 * under -fsanitize=address,undefined; any out-of-bounds access, leak or UB aborts the run.
 * Prints one checksum per routine (the pytest wrapper only checks the exit status). */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/pb_oracle.h"

static double checksum(const double* v, int64_t n) {
  double s = 0.0;
  for (int64_t i = 0; i < n; ++i) s += fabs(v[i]) * (double)(1 + i % 7);
  return s;
}

static double* vec(int64_t n) { return (double*)calloc((size_t)n, sizeof(double)); }

int main(void) {
  const int64_t shapes[][3] = {{3, 3, 3}, {5, 4, 3}, {8, 6, 10}, {16, 16, 16}, {7, 9, 4}};
  for (size_t s = 0; s < sizeof(shapes) / sizeof(shapes[0]); ++s) {
    const int64_t* n = shapes[s];
    const int64_t N = n[0] * n[1] * n[2];
    const double h[3] = {1.0 / n[0], 1.0 / n[1], 1.0 / n[2]};
    double *x = vec(N), *y = vec(N), *y2 = vec(N), *hist = vec(10002);
    pbo_fill_random(N, 20231015, 0, x);
    pbo_stencil_apply27(n, h, x, y);
    pbo_stencil_apply7(n, h, x, y2, 2);
    printf("stencil %lld %.17g %.17g\n", (long long)N, checksum(y, N), checksum(y2, N));
    for (int r = 1; r <= 3 && r <= n[2]; ++r) {
      pbo_assembled_apply(n, h, r, x, y2);
      printf("assembled r%d %.17g\n", r, checksum(y2, N));
    }
    const int64_t nl[3] = {n[0], n[1], n[2] - 1};
    pbo_stencil_slab(nl, h, x + n[0] * n[1], x, x + (n[2] - 1) * n[0] * n[1], y2);
    const int kinds[] = {0, 2, 3, 4};
    for (int pc = 0; pc <= 3; ++pc)
      for (size_t kk = 0; kk < sizeof(kinds) / sizeof(kinds[0]); ++kk) {
        if (pc >= 2 && (n[0] % 2 || n[1] % 2 || n[2] % 2)) continue;
        pbo_ksp_opts o;
        memset(&o, 0, sizeof(o));
        o.rtol = 1e-8;
        o.atol = 1e-50;
        o.dtol = 1e5;
        o.max_it = 300;
        o.pc_type = pc;
        o.nullspace = 1;
        o.op_kind = kinds[kk];
        o.nthreads = 1;
        o.mg_coarse_its = 4;
        o.omega = 1.0;
        o.nranks = 1;
        int64_t its = 0, nlog = 0;
        double* xs = vec(N);
        const int reason = pbo_cg_solve(n, h, &o, y, xs, hist, &its, &nlog);
        printf("cg pc%d op%d reason %d its %lld nlog %lld %.6g\n", pc, kinds[kk], reason,
               (long long)its, (long long)nlog, checksum(xs, N));
        free(xs);
      }
    double* work = vec(4 * N);
    printf("cg_fixed %.17g\n", pbo_cg_fixed(n, h, 5, 1, y, y2, work));
    free(work);
    if (n[0] % 2 == 0 && n[1] % 2 == 0 && n[2] % 2 == 0) {
      pbo_mg_apply(n, h, 3, 0, 4, 1.0, 1, x, y2);
      printf("mg %.17g levels %d\n", checksum(y2, N), pbo_mg_plan_levels(n, 1, 0));
      pbo_mg_apply(n, h, 2, 0, 1, 1.2, 1, x, y2);
      printf("sor %.17g\n", checksum(y2, N));
    }
    /* compact schemes (src/compact_schemes.f90) */
    double *f3 = vec(3 * N), *g3 = vec(3 * N);
    pbo_grad(n, x, h, f3);
    pbo_div(n, f3, h, y2);
    pbo_interp(n, x, y, -1);
    pbo_interp(n, y, y2, 1);
    pbo_lapl(n, x, h, g3);
    printf("compact %.17g %.17g %.17g\n", checksum(f3, 3 * N), checksum(y2, N), checksum(g3, N));
    free(f3);
    free(g3);
    free(x);
    free(y);
    free(y2);
    free(hist);
  }
  /* tridiagonal (src/tridsol.f90) and 1-D compact lines */
  for (int64_t m = 3; m <= 130; m += 31) {
    double *a = vec(m), *b = vec(m), *c = vec(m), *d = vec(m), *f = vec(m), *o = vec(m);
    for (int64_t i = 0; i < m; ++i) {
      a[i] = 0.3;
      b[i] = 1.0 + 0.01 * (double)i;
      c[i] = 0.25;
      d[i] = sin(0.1 * (double)i);
      f[i] = cos(0.2 * (double)i);
    }
    pbo_tdma(m, a, b, c, d);
    for (int64_t i = 0; i < m; ++i) b[i] = 1.0 + 0.01 * (double)i;
    pbo_tdma_periodic(m, a, b, c, d);
    pbo_grad_1d(m, f, 0.1, o, -1);
    pbo_interp_1d(m, f, o, 1);
    pbo_eval_1d_rhs(0.75, 0.05, 1, -1, m, f, o);
    printf("lines %lld %.17g %.17g\n", (long long)m, checksum(d, m), checksum(o, m));
    free(a); free(b); free(c); free(d); free(f); free(o);
  }
  printf("oracle_check ok\n");
  return 0;
}
