// bg_comm.cc -- the rule-table collective in the C ABI (include/bessgpu.h
// bg_comm_*, bg_em_allgather*): RCCL over xGMI, no torch.
//
// packets are independent, so no data-path collective; the only
// exchange is the ExactMatch table of a rule set too large to build on every
// GPU (C5, 1 M rules). Partition p of a sharded image holds the keys whose
// second hash selects it, and both candidate buckets of a key lie in its
// partition, so rank r can build partition r alone; one all-reduce (MAX) of
// the partition sizes fixes the layout, one all-gather assembles the image
// on every GPU. A bessd process with workers on several GPUs of a host uses
// bg_comm_init_all + bg_em_allgather_all (one thread, grouped calls); one
// process per GPU uses bg_comm_unique_id / bg_comm_init_rank and each rank
// calls bg_em_allgather.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>
#include <time.h>

#include <memory>
#include <vector>

#include "../../include/bessgpu.h"
#include "bg_internal.h"

using namespace bg;

struct bg_comm {
  ncclComm_t c = nullptr;
  int device = -1;
  int rank = 0, nranks = 1;
  // the last bg_em_allgather on this rank: ns in the size all-reduce, the
  // partition build (host), the upload + all-gather; image bytes
  uint64_t last_ns[3] = {0, 0, 0};
  uint64_t last_bytes = 0;
};

static uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

#define NCCL_TRY(expr)                                                        \
  do {                                                                        \
    ncclResult_t r_ = (expr);                                                 \
    if (r_ != ncclSuccess)                                                    \
      return fail(EIO, "%s: %s", #expr, ncclGetErrorString(r_));              \
  } while (0)

static_assert(NCCL_UNIQUE_ID_BYTES == BG_COMM_ID_BYTES, "bg_comm id size");

extern "C" {

int bg_comm_unique_id(uint8_t *id) {
  if (!id) return fail(EINVAL, "bad arguments");
  ncclUniqueId u;
  NCCL_TRY(ncclGetUniqueId(&u));
  memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

int bg_comm_init_rank(const uint8_t *id, int nranks, int rank, int device,
                      bg_comm **out) {
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(EINVAL, "bad arguments (rank %d of %d)", rank, nranks);
  if (int r = set_device(device)) return r;
  ncclUniqueId u;
  memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  std::unique_ptr<bg_comm> c(new bg_comm());
  NCCL_TRY(ncclCommInitRank(&c->c, nranks, u, rank));
  c->device = device;
  c->rank = rank;
  c->nranks = nranks;
  *out = c.release();
  return 0;
}

int bg_comm_init_all(const int *devices, int ndev, bg_comm **comms) {
  if (!devices || !comms || ndev < 1 || ndev > kMaxDevices)
    return fail(EINVAL, "bad arguments (%d devices)", ndev);
  std::vector<ncclComm_t> c((size_t)ndev);
  NCCL_TRY(ncclCommInitAll(c.data(), ndev, devices));
  for (int i = 0; i < ndev; i++) {
    comms[i] = new bg_comm();
    comms[i]->c = c[i];
    comms[i]->device = devices[i];
    comms[i]->rank = i;
    comms[i]->nranks = ndev;
  }
  return 0;
}

void bg_comm_destroy(bg_comm *c) {
  if (!c) return;
  if (c->c) (void)ncclCommDestroy(c->c);
  delete c;
}

int bg_comm_info(const bg_comm *c, int *rank, int *nranks, int *device) {
  if (!c) return fail(EINVAL, "bad arguments");
  if (rank) *rank = c->rank;
  if (nranks) *nranks = c->nranks;
  if (device) *device = c->device;
  return 0;
}

// One rank: its partition built here, the rest gathered from the others.
int bg_em_allgather(bg_em *em, bg_comm *comm, bg_stream_t stream) {
  if (!em || !comm) return fail(EINVAL, "bad arguments");
  const int nr = comm->nranks, rank = comm->rank;
  int r = set_device(comm->device);
  if (r) return r;
  hipStream_t s = (hipStream_t)stream;
  const uint64_t t0 = mono_ns();
  // the layout: the largest partition over all ranks (all-reduce MAX)
  uint64_t cnt = 0;
  if ((r = bg_em_part_count(em, rank, nr, &cnt))) return r;
  uint64_t *d_cnt = nullptr;
  HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_cnt), 8));
  std::unique_ptr<uint64_t, void (*)(uint64_t *)> cnt_guard(
      d_cnt, [](uint64_t *p) { (void)hipFree(p); });
  HIP_TRY(hipMemcpyAsync(d_cnt, &cnt, 8, hipMemcpyHostToDevice, s));
  NCCL_TRY(ncclAllReduce(d_cnt, d_cnt, 1, ncclUint64, ncclMax, comm->c, s));
  HIP_TRY(hipMemcpyAsync(&cnt, d_cnt, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  const uint64_t t1 = mono_ns();
  uint64_t part_bytes = 0;
  if ((r = bg_em_plan_count(em, nr, cnt, &part_bytes))) return r;
  // this rank's partition, in place in the gathered image
  std::vector<uint8_t> part(part_bytes);
  if ((r = bg_em_build_part(em, rank, part.data()))) return r;
  const uint64_t t2 = mono_ns();
  uint8_t *d_img = nullptr;
  HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_img), part_bytes * nr));
  uint8_t *mine = d_img + part_bytes * rank;
  hipError_t e = hipMemcpyAsync(mine, part.data(), part_bytes, hipMemcpyHostToDevice, s);
  ncclResult_t q = ncclSuccess;
  if (e == hipSuccess) q = ncclAllGather(mine, d_img, part_bytes, ncclUint8, comm->c, s);
  if (e == hipSuccess && q == ncclSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess || q != ncclSuccess) {
    (void)hipFree(d_img);
    return q != ncclSuccess ? fail(EIO, "ncclAllGather: %s", ncclGetErrorString(q))
                            : fail(EIO, "HIP: %s", hipGetErrorString(e));
  }
  const uint64_t t3 = mono_ns();
  comm->last_ns[0] = t1 - t0;
  comm->last_ns[1] = t2 - t1;
  comm->last_ns[2] = t3 - t2;
  comm->last_bytes = part_bytes * nr;
  return em_publish_owned(em, comm->device, d_img, part_bytes * nr);
}

int bg_comm_last_stats(const bg_comm *c, uint64_t *ns3, uint64_t *bytes) {
  if (!c) return fail(EINVAL, "bad arguments");
  if (ns3) memcpy(ns3, c->last_ns, sizeof(c->last_ns));
  if (bytes) *bytes = c->last_bytes;
  return 0;
}

// Every GPU of this process at once: the host holds all the rules, so each
// device gets its own partition uploaded and one grouped all-gather
// assembles the image on all of them.
int bg_em_allgather_all(bg_em *em, bg_comm *const *comms, int ncomm) {
  if (!em || !comms || ncomm < 1) return fail(EINVAL, "bad arguments");
  const int nr = comms[0]->nranks;
  if (ncomm != nr) return fail(EINVAL, "%d communicators for %d ranks", ncomm, nr);
  uint64_t part_bytes = 0;
  int r = bg_em_plan(em, nr, &part_bytes);
  if (r) return r;
  std::vector<uint8_t *> img((size_t)nr, nullptr);
  std::vector<hipStream_t> st((size_t)nr, nullptr);
  auto cleanup = [&]() {
    for (int i = 0; i < nr; i++) {
      if (st[i]) (void)hipStreamDestroy(st[i]);
      if (img[i]) (void)hipFree(img[i]);
    }
  };
  std::vector<uint8_t> part(part_bytes);
  for (int i = 0; i < nr && !r; i++) {
    const bg_comm *c = comms[i];
    if ((r = set_device(c->device))) break;
    if ((r = bg_em_build_part(em, c->rank, part.data()))) break;
    if (hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(reinterpret_cast<void **>(&img[i]), part_bytes * nr) != hipSuccess ||
        hipMemcpy(img[i] + part_bytes * c->rank, part.data(), part_bytes,
                  hipMemcpyHostToDevice) != hipSuccess)
      r = fail(EIO, "device %d: staging the partition failed", c->device);
  }
  if (r) {
    cleanup();
    return r;
  }
  ncclResult_t q = ncclGroupStart();
  for (int i = 0; i < nr && q == ncclSuccess; i++) {
    uint8_t *mine = img[i] + part_bytes * comms[i]->rank;
    q = ncclAllGather(mine, img[i], part_bytes, ncclUint8, comms[i]->c, st[i]);
  }
  ncclResult_t q2 = ncclGroupEnd();
  if (q == ncclSuccess) q = q2;
  for (int i = 0; i < nr && q == ncclSuccess; i++) {
    (void)hipSetDevice(comms[i]->device);
    if (hipStreamSynchronize(st[i]) != hipSuccess) q = ncclUnhandledCudaError;
  }
  if (q != ncclSuccess) {
    cleanup();
    return fail(EIO, "grouped ncclAllGather: %s", ncclGetErrorString(q));
  }
  for (int i = 0; i < nr; i++) {
    (void)hipSetDevice(comms[i]->device);
    (void)hipStreamDestroy(st[i]);
    st[i] = nullptr;
    r = em_publish_owned(em, comms[i]->device, img[i], part_bytes * nr);
    img[i] = nullptr;  // owned by the table now (or freed on failure)
    if (r) break;
  }
  cleanup();
  return r;
}

}  // extern "C"
