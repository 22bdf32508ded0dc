// Multi-GPU batch split for callers without torch.distributed ("the C ABI has no
// batch-split or collective entry points"). The Python path (distributed.py) runs the same protocol over
// torch.distributed: contiguous codeword ranges per rank, one setup broadcast of the code and tables from rank 0,
// one all-reduce of the counters per Eb/N0 point, no collective inside a decode.
//
// RCCL (NCCL's API on ROCm, over xGMI between the GPUs of a node) is opened at run time with dlopen: the
// 570-MB library is mapped only by a process that creates a communicator, and libibldpc.so itself keeps no
// link-time dependency on it (torch brings its own RCCL; two mappings of one library in one process are fine).
#include <dlfcn.h>

#include <cstring>
#include <mutex>
#include <string>

#include <rccl/rccl.h>

#include "common.h"
#include "ibldpc.h"

namespace {

int comm_fail(int code, const std::string& msg) { return ibl::set_error(code, msg.c_str()); }

// entry points typed from rccl.h's own declarations (a hand-written signature that drifts from the
// library's is an ABI mismatch no compiler sees through dlsym)
struct Rccl {
  void* so = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclBroadcast) bcast = nullptr;   // (sendbuff, recvbuff, count, type, root, comm, stream)
  decltype(&ncclAllReduce) allreduce = nullptr;
  decltype(&ncclGetErrorString) errstr = nullptr;
};

const Rccl* rccl(std::string* err) {
  static Rccl r;
  static std::once_flag once;
  static std::string why;
  std::call_once(once, [] {
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      r.so = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (r.so) break;
    }
    if (!r.so) {
      why = std::string("cannot load RCCL (librccl.so): ") + dlerror();
      return;
    }
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(r.so, "ncclGetUniqueId"));
    r.init_rank = reinterpret_cast<decltype(r.init_rank)>(dlsym(r.so, "ncclCommInitRank"));
    r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(r.so, "ncclCommDestroy"));
    r.bcast = reinterpret_cast<decltype(r.bcast)>(dlsym(r.so, "ncclBroadcast"));
    r.allreduce = reinterpret_cast<decltype(r.allreduce)>(dlsym(r.so, "ncclAllReduce"));
    r.errstr = reinterpret_cast<decltype(r.errstr)>(dlsym(r.so, "ncclGetErrorString"));
    if (!r.get_unique_id || !r.init_rank || !r.destroy || !r.bcast || !r.allreduce || !r.errstr)
      why = "RCCL lacks an entry point this library needs";
  });
  if (!why.empty()) {
    *err = why;
    return nullptr;
  }
  return &r;
}

}  // namespace

struct ibl_comm {
  const Rccl* r = nullptr;
  ncclComm_t comm = nullptr;
  int device = 0, nranks = 1, rank = 0;
};

static_assert(sizeof(ncclUniqueId) == IBL_COMM_ID_BYTES, "ncclUniqueId size");

#define NCCLCHK(c, expr)                                                                    \
  do {                                                                                      \
    ncclResult_t _r = (expr);                                                               \
    if (_r != ncclSuccess) return comm_fail(IBL_EHIP, std::string(#expr) + ": " + (c)->errstr(_r)); \
  } while (0)

extern "C" {

int ibl_shard_range(int64_t total, int32_t rank, int32_t world, int64_t* start, int64_t* count) {
  if (!start || !count || total < 0 || world < 1 || rank < 0 || rank >= world)
    return comm_fail(IBL_EINVAL, "ibl_shard_range: need total >= 0, 0 <= rank < world");
  const int64_t base = total / world, extra = total % world;
  *start = (int64_t)rank * base + (rank < extra ? rank : extra);
  *count = base + (rank < extra ? 1 : 0);
  return IBL_OK;
}

int ibl_comm_unique_id(uint8_t* id) {
  if (!id) return comm_fail(IBL_EINVAL, "id is NULL");
  std::string err;
  const Rccl* r = rccl(&err);
  if (!r) return comm_fail(IBL_EUNSUPPORTED, err);
  ncclUniqueId u;
  NCCLCHK(r, r->get_unique_id(&u));
  std::memcpy(id, &u, sizeof(u));
  return IBL_OK;
}

int ibl_comm_create(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device, ibl_comm** out) {
  if (!out) return comm_fail(IBL_EINVAL, "out is NULL");
  *out = nullptr;
  if (!id || nranks < 1 || rank < 0 || rank >= nranks) return comm_fail(IBL_EINVAL, "need an id and 0 <= rank < nranks");
  std::string err;
  const Rccl* r = rccl(&err);
  if (!r) return comm_fail(IBL_EUNSUPPORTED, err);
  if (hipSetDevice(device) != hipSuccess) return comm_fail(IBL_EHIP, "hipSetDevice failed");
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  auto* c = new ibl_comm();
  c->r = r;
  c->device = device;
  c->nranks = nranks;
  c->rank = rank;
  const ncclResult_t rc = r->init_rank(&c->comm, nranks, u, rank);
  if (rc != ncclSuccess) {
    delete c;
    return comm_fail(IBL_EHIP, std::string("ncclCommInitRank: ") + r->errstr(rc));
  }
  *out = c;
  return IBL_OK;
}

int ibl_comm_broadcast(ibl_comm* c, void* d_buf, int64_t bytes, int32_t root, void* stream) {
  if (!c || (!d_buf && bytes > 0) || bytes < 0 || root < 0 || root >= c->nranks)
    return comm_fail(IBL_EINVAL, "bad broadcast arguments");
  if (hipSetDevice(c->device) != hipSuccess) return comm_fail(IBL_EHIP, "hipSetDevice failed");
  NCCLCHK(c->r, c->r->bcast(d_buf, d_buf, (size_t)bytes, ncclUint8, root, c->comm, (hipStream_t)stream));
  return IBL_OK;
}

int ibl_comm_allreduce_sum_i64(ibl_comm* c, int64_t* d_buf, int64_t count, void* stream) {
  if (!c || (!d_buf && count > 0) || count < 0) return comm_fail(IBL_EINVAL, "bad all-reduce arguments");
  if (hipSetDevice(c->device) != hipSuccess) return comm_fail(IBL_EHIP, "hipSetDevice failed");
  NCCLCHK(c->r, c->r->allreduce(d_buf, d_buf, (size_t)count, ncclInt64, ncclSum, c->comm, (hipStream_t)stream));
  return IBL_OK;
}

void ibl_comm_destroy(ibl_comm* c) {
  if (!c) return;
  if (c->comm) (void)c->r->destroy(c->comm);
  delete c;
}

}  // extern "C"
