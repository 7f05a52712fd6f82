// host_check.cpp -- host sanitizer driver for the host logic of libpoissbox_gpu
// (pb_runtime.cpp, pb_solver.cpp) built with -fsanitize=address,undefined on the host side only.
// Runs without a GPU: option parsing, slab partition, argument validation and the error paths
// of every entry point that must fail cleanly (no device, NULL handles) -- the code a caller
// reaches before any kernel launches. Exit status 0 = clean.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "poissbox_gpu.h"

static int fails = 0;
#define EXPECT(cond)                                                    \
  do {                                                                  \
    if (!(cond)) {                                                      \
      std::fprintf(stderr, "FAILED %s:%d %s\n", __FILE__, __LINE__, #cond); \
      ++fails;                                                          \
    }                                                                   \
  } while (0)

int main() {
  int ma = -1, mi = -1;
  EXPECT(pb_version(&ma, &mi) == PB_OK && ma == PB_VERSION_MAJOR && mi == PB_VERSION_MINOR);
  // slab partition: README.md:30-32's 64^3 on 3 ranks = 22/21/21 planes, and every split covers
  // [0, nz) exactly once
  int64_t k0 = 0, nk = 0;
  for (int64_t nz = 1; nz <= 70; ++nz)
    for (int R = 1; R <= 9; ++R) {
      int64_t next = 0;
      for (int r = 0; r < R; ++r) {
        EXPECT(pb_slab_partition(nz, R, r, &k0, &nk) == PB_OK);
        EXPECT(k0 == next);
        next = k0 + nk;
      }
      EXPECT(next == nz);
    }
  EXPECT(pb_slab_partition(64, 3, 0, &k0, &nk) == PB_OK && nk == 22);
  EXPECT(pb_slab_partition(0, 3, 0, &k0, &nk) == PB_ERR_ARG);
  EXPECT(pb_slab_partition(8, 2, 2, &k0, &nk) == PB_ERR_ARG);
  EXPECT(std::strlen(pb_last_error()) > 0);

  // options database
  pb_ksp_opts o;
  EXPECT(pb_ksp_opts_default(&o) == PB_OK && o.rtol == 1e-5 && o.max_it == 10000);
  const std::vector<std::vector<std::string>> argvs = {
      {"-ksp_type", "cg", "-pc_type", "jacobi", "-ksp_rtol", "1e-10", "-ksp_monitor"},
      {"-pc_type", "mg", "-pc_mg_levels", "5", "-pc_mg_coarse_its", "3", "-pc_sor_omega", "1.3"},
      {"-pc_type", "gamg", "-mg_coarse_ksp_max_it", "2", "-ksp_converged_reason"},
      {"-pc_type", "none", "-ksp_atol", "1e-30", "-ksp_divtol", "1e9", "-ksp_max_it", "77"},
      {"-ksp_rtol"},  // missing value: ignored
      {std::string(4096, 'x'), "-pc_type", "sor"},
      {}};
  for (const auto& a : argvs) {
    std::vector<const char*> v;
    for (const auto& s : a) v.push_back(s.c_str());
    pb_ksp_opts_default(&o);
    EXPECT(pb_ksp_opts_parse(&o, (int)v.size(), v.data()) == PB_OK);
  }
  {
    const char* bad[] = {"-pc_type", "ilu"};
    EXPECT(pb_ksp_opts_parse(&o, 2, bad) == PB_ERR_UNSUPPORTED);
    const char* bad2[] = {"-ksp_type", "gmres"};
    EXPECT(pb_ksp_opts_parse(&o, 2, bad2) == PB_ERR_UNSUPPORTED);
    EXPECT(pb_ksp_opts_parse(nullptr, 0, nullptr) == PB_ERR_ARG);
  }
  {
    const char* v[] = {"-pc_type", "mg", "-pc_mg_levels", "4", "-ksp_max_it", "123"};
    pb_ksp_opts_default(&o);
    EXPECT(pb_ksp_opts_parse(&o, 6, v) == PB_OK && o.pc_type == PB_PC_MG && o.mg_levels == 4 &&
           o.max_it == 123);
  }

  // no GPU in the CPU tier: context creation must fail cleanly, never crash
  pb_ctx* ctx = nullptr;
  const int rc = pb_ctx_create(0, 0, 1, nullptr, &ctx);
  if (rc == PB_OK) {  // (a GPU is present: exercise create/destroy instead)
    EXPECT(pb_ctx_destroy(ctx) == PB_OK);
  } else {
    EXPECT(rc == PB_ERR_ARG || rc == PB_ERR_HIP);
    EXPECT(ctx == nullptr);
  }
  EXPECT(pb_ctx_create(0, 2, 2, nullptr, &ctx) == PB_ERR_ARG || rc != PB_OK);
  EXPECT(pb_ctx_create(0, 0, 1, nullptr, nullptr) == PB_ERR_ARG);

  // NULL handles: argument errors (or no-ops for destroy), never a dereference
  double d = 0.0;
  int64_t i64 = 0;
  int iv = 0;
  EXPECT(pb_ctx_sync(nullptr) == PB_ERR_ARG);
  EXPECT(pb_ctx_barrier(nullptr) == PB_ERR_ARG);
  EXPECT(pb_ctx_comm_status(nullptr, &iv) == PB_ERR_ARG);
  EXPECT(pb_ctx_get_rank(nullptr, &iv, &iv) == PB_ERR_ARG);
  EXPECT(pb_ctx_set_timing(nullptr, 1) == PB_ERR_ARG);
  EXPECT(pb_ctx_get_timing(nullptr, "stencil", &d, &i64) == PB_ERR_ARG);
  EXPECT(pb_ctx_reset_timing(nullptr) == PB_ERR_ARG);
  EXPECT(pb_ctx_set_host_transport(nullptr, nullptr, nullptr, nullptr) == PB_ERR_ARG);
  EXPECT(pb_ctx_destroy(nullptr) == PB_OK);
  const int64_t n3[3] = {8, 8, 8};
  pb_grid* g = nullptr;
  EXPECT(pb_grid_create(nullptr, n3, nullptr, &g) == PB_ERR_ARG);
  EXPECT(pb_grid_get_corners(nullptr, nullptr, nullptr) == PB_ERR_ARG);
  EXPECT(pb_grid_get_info(nullptr, nullptr, nullptr, nullptr) == PB_ERR_ARG);
  EXPECT(pb_grid_destroy(nullptr) == PB_OK);
  pb_vec* v = nullptr;
  EXPECT(pb_vec_create(nullptr, &v) == PB_ERR_ARG);
  EXPECT(pb_vec_duplicate(nullptr, &v) == PB_ERR_ARG);
  EXPECT(pb_vec_set(nullptr, 1.0) == PB_ERR_ARG);
  EXPECT(pb_vec_copy(nullptr, nullptr) == PB_ERR_ARG);
  EXPECT(pb_vec_axpy(nullptr, 1.0, nullptr) == PB_ERR_ARG);
  EXPECT(pb_vec_aypx(nullptr, 1.0, nullptr) == PB_ERR_ARG);
  EXPECT(pb_vec_scale(nullptr, 1.0) == PB_ERR_ARG);
  EXPECT(pb_vec_dot(nullptr, nullptr, &d) == PB_ERR_ARG);
  EXPECT(pb_vec_norm2(nullptr, &d) == PB_ERR_ARG);
  EXPECT(pb_vec_sum(nullptr, &d) == PB_ERR_ARG);
  EXPECT(pb_vec_set_values_host(nullptr, &d) == PB_ERR_ARG);
  EXPECT(pb_vec_get_values_host(nullptr, &d) == PB_ERR_ARG);
  EXPECT(pb_vec_set_random(nullptr, 1) == PB_ERR_ARG);
  EXPECT(pb_vec_device_ptr(nullptr, nullptr, nullptr) == PB_ERR_ARG);
  EXPECT(pb_vec_destroy(nullptr) == PB_OK);
  pb_op* op = nullptr;
  EXPECT(pb_op_create(nullptr, PB_OP_STAR7, nullptr, &op) == PB_ERR_ARG);
  EXPECT(pb_op_apply(nullptr, nullptr, nullptr) == PB_ERR_ARG);
  EXPECT(pb_op_get_diagonal(nullptr, &d) == PB_ERR_ARG);
  EXPECT(pb_op_get_ownership_range(nullptr, &i64, &i64) == PB_ERR_ARG);
  EXPECT(pb_op_destroy(nullptr) == PB_OK);
  pb_ksp* k = nullptr;
  EXPECT(pb_ksp_create(nullptr, nullptr, &o, &k) == PB_ERR_ARG);
  EXPECT(pb_ksp_iterate(nullptr, 1) == PB_ERR_ARG);
  EXPECT(pb_ksp_begin(nullptr, nullptr, nullptr) == PB_ERR_ARG);
  EXPECT(pb_ksp_end(nullptr, nullptr, nullptr, 0) == PB_ERR_ARG);
  EXPECT(pb_ksp_pc_apply(nullptr, nullptr, nullptr) == PB_ERR_ARG);
  EXPECT(pb_ksp_pc_levels(nullptr, &iv) == PB_ERR_ARG);
  EXPECT(pb_ksp_destroy(nullptr) == PB_OK);
  std::printf("host_check %s (%d failures)\n", fails ? "FAILED" : "ok", fails);
  return fails ? 1 : 0;
}
