// comm.cpp — the multi-GPU counter all-reduce over RCCL (xGMI), the only
// collective of the path (the reference's per-thread counters are
// summed under a mutex, lib/lab/src/threadsafe_sourcesink.cc).
//
// The product library talks to RCCL itself, on the context's own HIP stream
// and through the same HIP runtime as its kernels: the Python drivers use
// torch.distributed (gloo) only for rendezvous and CPU control (barriers, the
// unique id's broadcast, the timing gather).  librccl is opened on first use
// (dlopen), so a host without it, or a single-GPU run, never loads it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "comm.hpp"

namespace kml {

namespace {

struct RcclApi {
  bool tried = false, ok = false;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::string why, path;
};

// The directory of the HIP runtime this library's kernels run on (the first
// libamdhip64.so.7 the process loaded: /opt/rocm's when the library is loaded
// before torch, torch's bundled copy otherwise).
std::string hip_runtime_path(const void *fn) {
  Dl_info info{};
  if (!dladdr(fn, &info) || !info.dli_fname) return "";
  return info.dli_fname;
}

std::string dir_of(const std::string &p) {
  const size_t k = p.rfind('/');
  return k == std::string::npos ? std::string() : p.substr(0, k + 1);
}

RcclApi &api() {
  static RcclApi a;
  if (a.tried) return a;
  a.tried = true;
  // librccl must run on the SAME HIP runtime as the library's streams.  Two
  // runtimes can be mapped into one process (the library's /opt/rocm copy and
  // torch's bundled one), and both librccl copies have the soname
  // librccl.so.1, so dlopen("librccl.so.1") hands back whichever is already
  // loaded (torch's, bound to torch's runtime: "unhandled cuda error" on the
  // library's stream).  Open the librccl next to our runtime by path, then
  // check what its HIP symbols resolve to.
  const std::string ours = hip_runtime_path(reinterpret_cast<const void *>(&hipStreamSynchronize));
  const std::string dir = dir_of(ours);
  void *h = nullptr;
  for (const std::string &cand : {dir + "librccl.so.1", dir + "librccl.so", std::string("/opt/rocm/lib/librccl.so.1")}) {
    if (cand.empty() || cand[0] != '/') continue;
    h = dlopen(cand.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!h) continue;
    const void *theirs = dlsym(h, "hipStreamSynchronize");
    if (theirs && hip_runtime_path(theirs) == ours) {
      a.path = cand;
      break;
    }
    a.why += cand + " is bound to HIP runtime " + (theirs ? hip_runtime_path(theirs) : std::string("?")) +
             ", the library runs on " + ours + "; ";
    dlclose(h);
    h = nullptr;
  }
  if (!h) {
    a.why = "no librccl bound to the library's HIP runtime (" + ours + "): " + a.why;
    return a;
  }
  a.get_unique_id = reinterpret_cast<decltype(a.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
  a.init_rank = reinterpret_cast<decltype(a.init_rank)>(dlsym(h, "ncclCommInitRank"));
  a.all_reduce = reinterpret_cast<decltype(a.all_reduce)>(dlsym(h, "ncclAllReduce"));
  a.destroy = reinterpret_cast<decltype(a.destroy)>(dlsym(h, "ncclCommDestroy"));
  a.error_string = reinterpret_cast<decltype(a.error_string)>(dlsym(h, "ncclGetErrorString"));
  a.ok = a.get_unique_id && a.init_rank && a.all_reduce && a.destroy && a.error_string;
  if (!a.ok) a.why = a.path + " lacks an NCCL entry point";
  return a;
}

std::string nccl_err(ncclResult_t r) {
  return api().error_string ? api().error_string(r) : ("ncclResult " + std::to_string((int)r));
}

}  // namespace

struct RcclComm {
  ncclComm_t comm = nullptr;
  int world = 0, rank = 0;
};

static_assert(sizeof(ncclUniqueId) == kCommIdBytes, "RCCL unique id size");

int rccl_unique_id(unsigned char *out, std::string &err) {
  RcclApi &a = api();
  if (!a.ok) {
    err = a.why;
    return -1;
  }
  ncclUniqueId id;
  const ncclResult_t r = a.get_unique_id(&id);
  if (r != ncclSuccess) {
    err = "ncclGetUniqueId: " + nccl_err(r);
    return -1;
  }
  memcpy(out, id.internal, kCommIdBytes);
  return 0;
}

RcclComm *rccl_init(const unsigned char *id, int world, int rank, std::string &err) {
  RcclApi &a = api();
  if (!a.ok) {
    err = a.why;
    return nullptr;
  }
  ncclUniqueId uid;
  memcpy(uid.internal, id, kCommIdBytes);
  RcclComm *c = new RcclComm;
  c->world = world;
  c->rank = rank;
  const ncclResult_t r = a.init_rank(&c->comm, world, uid, rank);  // collective over the world's ranks
  if (r != ncclSuccess) {
    err = "ncclCommInitRank (" + a.path + "): " + nccl_err(r);
    delete c;
    return nullptr;
  }
  return c;
}

int rccl_allreduce(RcclComm *c, void *buf, size_t n, bool f64, hipStream_t s, std::string &err) {
  const ncclResult_t r = api().all_reduce(buf, buf, n, f64 ? ncclFloat64 : ncclUint64, ncclSum, c->comm, s);
  if (r != ncclSuccess) {
    err = "ncclAllReduce: " + nccl_err(r);
    return -1;
  }
  return 0;
}

int rccl_size(const RcclComm *c) { return c ? c->world : 0; }

void rccl_destroy(RcclComm *c) {
  if (!c) return;
  if (c->comm) api().destroy(c->comm);
  delete c;
}

}  // namespace kml
