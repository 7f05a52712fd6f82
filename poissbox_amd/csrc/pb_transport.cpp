// pb_transport.cpp -- launcher-agnostic multi-process start (≙ MPI_Init + MPI_Comm_rank/size,
// src/example.f90:43-47) and the built-in shared-memory host transport.
//
// pb_ctx_create_from_env reads the rank layout any common launcher exports (torchrun: RANK /
// WORLD_SIZE / LOCAL_RANK; Open MPI: OMPI_COMM_WORLD_*; PMI: PMI_RANK / PMI_SIZE), so a Fortran or
// C driver runs unchanged under `torchrun --no-python`, `mpirun` or a plain fork. Two transports:
//  * rccl (default when every rank has its own GPU): rank 0's RCCL unique id travels through a
//    file in PB_RENDEZVOUS_DIR (default /tmp) keyed by the job (PB_JOB_ID, else MASTER_PORT),
//    written atomically (write + rename) and removed once the communicator is up;
//  * shm (default when ranks outnumber the visible GPUs, or PB_TRANSPORT=shm): halo planes and
//    scalar sums through a POSIX shared-memory segment with a spinning process-shared barrier.
//    Ranks may share one GPU (RCCL refuses that), which is how the multi-rank Fortran demo runs on
//    a one-GPU box. Every barrier wait is bounded by the context's PB_COMM_TIMEOUT_MS.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>

#include "pb_internal.hpp"

namespace pb {

namespace {

int env_first(const char* const* names, int dflt) {
  for (const char* const* n = names; *n; ++n) {
    const char* v = getenv(*n);
    if (v && *v) return atoi(v);
  }
  return dflt;
}

std::string sanitized(const char* v) {
  std::string s(v);
  for (char& c : s)
    if (!isalnum((unsigned char)c)) c = '_';
  return s;
}

// The rendezvous name of this launch: the job (PB_JOB_ID, else the launcher's port / job id) plus
// torchrun's restart count, so an elastic restart on the same MASTER_PORT never meets the files
// of the attempt before it.
std::string job_key() {
  const char* names[] = {"PB_JOB_ID", "MASTER_PORT", "OMPI_MCA_ess_base_jobid", "PMI_JOBID",
                         nullptr};
  std::string key = "default";
  for (const char* const* n = names; *n; ++n) {
    const char* v = getenv(*n);
    if (v && *v) {
      key = sanitized(v);
      break;
    }
  }
  const char* rc = getenv("TORCHELASTIC_RESTART_COUNT");
  if (rc && *rc) key += "_r" + sanitized(rc);
  return key;
}

// Wall-clock start of this process (seconds since the epoch): /proc/self/stat's start time in
// clock ticks after boot plus /proc/stat's btime. 0 if unavailable.
double process_start_epoch_s() {
  double boot = 0.0;
  if (FILE* f = fopen("/proc/stat", "r")) {
    char line[256];
    while (fgets(line, sizeof line, f))
      if (!strncmp(line, "btime ", 6)) boot = atof(line + 6);
    fclose(f);
  }
  unsigned long long ticks = 0;
  if (FILE* f = fopen("/proc/self/stat", "r")) {
    char buf[1024];
    const size_t n = fread(buf, 1, sizeof buf - 1, f);
    fclose(f);
    buf[n] = '\0';
    const char* p = strrchr(buf, ')');  // the command name may contain spaces
    for (int field = 2; p && *p && field < 22; ++p)
      if (*p == ' ') ++field;
    if (p) ticks = strtoull(p, nullptr, 10);
  }
  const long hz = sysconf(_SC_CLK_TCK);
  if (boot <= 0.0 || !ticks || hz <= 0) return 0.0;
  return boot + (double)ticks / (double)hz;
}

// A rendezvous object (uid file, shm segment) last written before this launch began belongs to
// an earlier run that died before cleaning up: ignore it. "Before this launch" = more than
// PB_RENDEZVOUS_SLACK_S (default 120) before this process started (the ranks of one launch start
// within that of each other).
int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// ... unless this rank has already waited longer than the slack itself: a rank that
// starts more than the slack after rank 0 (slow container start, staggered scheduler, a clock
// that disagrees with the file system's) then takes the file it sees, with a warning -- at worst
// a stale id, which the bounded communicator init reports as PB_ERR_COMM. `waited_ms`: how long
// the caller has been waiting for this object; `what` names it in the log line (once per object).
bool fresh_enough(const struct stat& st, int64_t waited_ms, const char* what) {
  static const double start = process_start_epoch_s();
  if (start <= 0.0) return true;
  const double slack = std::max(0, env_int("PB_RENDEZVOUS_SLACK_S", 120));
  const double mtime = (double)st.st_mtim.tv_sec + 1e-9 * (double)st.st_mtim.tv_nsec;
  if (mtime >= start - slack) return true;
  static std::string logged;
  const bool accept = (double)waited_ms > 1000.0 * slack;
  if (logged != std::string(what) + (accept ? "+" : "-")) {
    logged = std::string(what) + (accept ? "+" : "-");
    fprintf(stderr, "[poissbox] rendezvous: %s was written %.0f s before this process started "
            "(PB_RENDEZVOUS_SLACK_S %.0f): %s\n", what, start - mtime, slack,
            accept ? "accepted after waiting the slack out" : "ignored as stale for now");
  }
  return accept;
}

void nap() {
  timespec ts{0, 20000};
  nanosleep(&ts, nullptr);
}

// ---- shared-memory transport ----
struct ShmHdr {
  std::atomic<int> ready;
  std::atomic<int> joined;
  std::atomic<int> count;
  std::atomic<int> gen;
  int nranks;
  int64_t cap;  // doubles per plane slot
};
static_assert(std::atomic<int>::is_always_lock_free, "process-shared atomics");

struct Shm {
  ShmHdr* hdr = nullptr;
  double* data = nullptr;  // per rank: [lo (cap) | hi (cap) | red (64)]
  size_t bytes = 0;
  int rank = 0, nranks = 1;
  int64_t timeout_ms = 180000;
  double* slot(int r) const { return data + (size_t)r * (2 * hdr->cap + 64); }
};

int shm_barrier(Shm* s) {
  ShmHdr* h = s->hdr;
  const int g = h->gen.load(std::memory_order_acquire);
  if (h->count.fetch_add(1, std::memory_order_acq_rel) == s->nranks - 1) {
    h->count.store(0, std::memory_order_relaxed);
    h->gen.fetch_add(1, std::memory_order_release);
    return 0;
  }
  const int64_t t0 = now_ms();
  for (int64_t spin = 0; h->gen.load(std::memory_order_acquire) == g; ++spin) {
    if (spin > 2048) nap();
    if ((spin & 255) == 255 && now_ms() - t0 > s->timeout_ms) return 1;  // a peer is gone
  }
  return 0;
}

int shm_sendrecv(void* user, const double* s_lo, const double* s_hi, double* r_lo, double* r_hi,
                 int64_t count) {
  Shm* s = (Shm*)user;
  const int down = (s->rank + s->nranks - 1) % s->nranks, up = (s->rank + 1) % s->nranks;
  const int64_t cap = s->hdr->cap;
  for (int64_t off = 0; off < count; off += cap) {  // planes larger than a slot go in pieces
    const int64_t m = std::min(cap, count - off);
    double* mine = s->slot(s->rank);
    memcpy(mine, s_lo + off, (size_t)m * sizeof(double));
    memcpy(mine + cap, s_hi + off, (size_t)m * sizeof(double));
    if (shm_barrier(s)) return 1;
    memcpy(r_lo + off, s->slot(down) + cap, (size_t)m * sizeof(double));  // plane below me
    memcpy(r_hi + off, s->slot(up), (size_t)m * sizeof(double));          // plane above me
    if (shm_barrier(s)) return 1;
  }
  return 0;
}

int shm_allreduce(void* user, double* vals, int count) {
  Shm* s = (Shm*)user;
  for (int off = 0; off < count; off += 64) {
    const int m = std::min(64, count - off);
    double* red = s->slot(s->rank) + 2 * s->hdr->cap;
    memcpy(red, vals + off, (size_t)m * sizeof(double));
    if (shm_barrier(s)) return 1;
    for (int e = 0; e < m; ++e) {  // rank order: every rank sums identically
      double t = 0.0;
      for (int r = 0; r < s->nranks; ++r) t += (s->slot(r) + 2 * s->hdr->cap)[e];
      vals[off + e] = t;
    }
    if (shm_barrier(s)) return 1;
  }
  return 0;
}

int shm_attach(pb_ctx* ctx, const std::string& key, Shm** out) {
  const std::string name = "/pb_shm_" + key;
  const int64_t cap = std::max(1024, env_int("PB_SHM_SLOT_DOUBLES", 1 << 18));
  const int P = ctx->nranks;
  const size_t bytes = 4096 + (size_t)P * (2 * cap + 64) * sizeof(double);
  Shm* s = new Shm();
  s->rank = ctx->rank;
  s->nranks = P;
  s->timeout_ms = ctx->comm_timeout_ms;
  s->bytes = bytes;
  int fd = -1;
  const int64_t t0 = now_ms();
  if (ctx->rank == 0) {
    shm_unlink(name.c_str());  // a stale segment of a crashed run with the same key
    fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, (off_t)bytes) != 0) {
      if (fd >= 0) close(fd);
      delete s;
      return set_error(PB_ERR_COMM, "shm transport: cannot create %s (%s)", name.c_str(),
                       strerror(errno));
    }
  } else {
    for (;;) {  // rank 0 creates the segment and sizes it; wait for both
      fd = shm_open(name.c_str(), O_RDWR, 0600);
      struct stat st;
      if (fd >= 0 && fstat(fd, &st) == 0 && (size_t)st.st_size == bytes &&
          fresh_enough(st, now_ms() - t0, name.c_str()))
        break;
      if (fd >= 0) close(fd);
      fd = -1;
      if (now_ms() - t0 > ctx->comm_timeout_ms) {
        delete s;
        return set_error(PB_ERR_COMM, "shm transport: %s never appeared", name.c_str());
      }
      nap();
    }
  }
  void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) {
    delete s;
    return set_error(PB_ERR_COMM, "shm transport: mmap failed (%s)", strerror(errno));
  }
  s->hdr = (ShmHdr*)m;
  s->data = (double*)((char*)m + 4096);
  if (ctx->rank == 0) {
    s->hdr->nranks = P;
    s->hdr->cap = cap;
    s->hdr->count.store(0);
    s->hdr->gen.store(0);
    s->hdr->joined.store(0);
    s->hdr->ready.store(1, std::memory_order_release);
  } else {
    while (s->hdr->ready.load(std::memory_order_acquire) != 1) {
      if (now_ms() - t0 > ctx->comm_timeout_ms) {
        munmap(m, bytes);
        delete s;
        return set_error(PB_ERR_COMM, "shm transport: segment never initialised");
      }
      nap();
    }
  }
  s->hdr->joined.fetch_add(1);
  if (shm_barrier(s)) {
    munmap(m, bytes);
    delete s;
    shm_unlink(name.c_str());  // leave nothing behind in /dev/shm
    return set_error(PB_ERR_COMM, "shm transport: not every rank joined within %lld ms",
                     (long long)ctx->comm_timeout_ms);
  }
  if (ctx->rank == 0) shm_unlink(name.c_str());  // everyone is mapped: nothing left in /dev/shm
  *out = s;
  return PB_OK;
}

// ---- RCCL unique id through a rendezvous file ----
int uid_rendezvous(int rank, const std::string& key, unsigned char uid[128], int64_t timeout_ms,
                   std::string* path_out) {
  const char* dir = getenv("PB_RENDEZVOUS_DIR");
  const std::string path = std::string(dir && *dir ? dir : "/tmp") + "/pb_uid_" + key;
  *path_out = path;
  if (rank == 0) {
    PB_TRY(pb_comm_unique_id(uid));
    const std::string tmp = path + ".tmp" + std::to_string((long)getpid());
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f || fwrite(uid, 1, 128, f) != 128) {
      if (f) fclose(f);
      return set_error(PB_ERR_COMM, "rendezvous: cannot write %s", tmp.c_str());
    }
    fclose(f);
    if (rename(tmp.c_str(), path.c_str()) != 0)
      return set_error(PB_ERR_COMM, "rendezvous: cannot publish %s", path.c_str());
    return PB_OK;
  }
  const int64_t t0 = now_ms();
  for (;;) {
    FILE* f = fopen(path.c_str(), "rb");
    if (f) {
      struct stat st;
      const bool fresh = fstat(fileno(f), &st) == 0 && fresh_enough(st, now_ms() - t0, path.c_str());
      const size_t got = fresh ? fread(uid, 1, 128, f) : 0;
      fclose(f);
      if (got == 128) return PB_OK;
    }
    if (now_ms() - t0 > timeout_ms)
      return set_error(PB_ERR_COMM, "rendezvous: %s never appeared (rank 0 missing?)",
                       path.c_str());
    nap();
  }
}

}  // namespace

void transport_destroy(pb_ctx* ctx) {
  if (!ctx->shm) return;
  Shm* s = (Shm*)ctx->shm;
  munmap((void*)s->hdr, s->bytes);
  delete s;
  ctx->shm = nullptr;
}

}  // namespace pb

using namespace pb;

extern "C" {

int pb_ctx_create_from_env(int device, pb_ctx** out) {
  PB_CHECK_ARG(out, "ctx out is NULL");
  const char* rank_names[] = {"RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", nullptr};
  const char* size_names[] = {"WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", nullptr};
  const char* local_names[] = {"LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID",
                               nullptr};
  const int rank = env_first(rank_names, 0);
  const int world = env_first(size_names, 1);
  const int local = env_first(local_names, rank);
  PB_CHECK_ARG(world >= 1 && rank >= 0 && rank < world, "bad rank / world size in the environment");
  int ndev = 0;
  PB_HIP(hipGetDeviceCount(&ndev));
  PB_CHECK_ARG(ndev > 0, "no GPU visible");
  int dev = env_int("PB_DEVICE", -1);
  if (dev < 0) dev = world == 1 && device >= 0 ? device : local % ndev;
  if (world == 1) return pb_ctx_create(dev, 0, 1, nullptr, out);
  const char* tr = getenv("PB_TRANSPORT");
  const bool shm = tr && *tr ? !strcmp(tr, "shm") : world > ndev;
  if (tr && *tr && strcmp(tr, "shm") && strcmp(tr, "rccl"))
    return set_error(PB_ERR_ARG, "PB_TRANSPORT=%s: rccl or shm", tr);
  const std::string key = job_key();
  if (shm) {
    pb_ctx* ctx = nullptr;
    PB_TRY(pb_ctx_create(dev, rank, world, nullptr, &ctx));
    Shm* s = nullptr;
    int rc = shm_attach(ctx, key, &s);
    if (rc == PB_OK) {
      ctx->shm = s;
      rc = pb_ctx_set_host_transport(ctx, shm_sendrecv, shm_allreduce, s);
    }
    if (rc != PB_OK) {
      pb_ctx_destroy(ctx);
      return rc;
    }
    *out = ctx;
    return PB_OK;
  }
  unsigned char uid[128];
  std::string path;
  const int64_t timeout = std::max(1, env_int("PB_COMM_TIMEOUT_MS", 180000));
  PB_TRY(uid_rendezvous(rank, key, uid, timeout, &path));
  const int rc = pb_ctx_create(dev, rank, world, uid, out);  // collective: all ranks joined
  if (rank == 0) unlink(path.c_str());
  return rc;
}

int pb_ctx_allreduce_host(pb_ctx* ctx, double* vals, int count) {
  PB_CHECK_ARG(ctx && vals && count >= 0 && count <= 32, "bad allreduce args (count <= 32)");
  if (!ctx->split || count == 0) return PB_OK;
  double* d = ctx->d_scalars + 32;  // the barrier slot region (pb_ctx_barrier uses [32])
  PB_HIP(hipMemcpyAsync(d, vals, (size_t)count * sizeof(double), hipMemcpyHostToDevice,
                        ctx->stream));
  PB_TRY(allreduce_device(ctx, d, count));
  PB_HIP(hipMemcpyAsync(ctx->h_scalars + 32, d, (size_t)count * sizeof(double),
                        hipMemcpyDeviceToHost, ctx->stream));
  PB_SYNC(ctx, "pb_ctx_allreduce_host");
  memcpy(vals, ctx->h_scalars + 32, (size_t)count * sizeof(double));
  return PB_OK;
}

}  // extern "C"
