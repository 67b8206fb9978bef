// gather.hip -- the multi-GPU gather of the tile-sharded encode as C-ABI entry
// points over RCCL (SURVEY.md section 8(b) "hic_gather_*"): an RCCL communicator
// (one rank per GPU) and a variable-size gather of every rank's slice of a
// whole-image buffer into one rank, posted as ONE RCCL group of sends and
// receives on the caller's stream.  Several gathers (different roots, e.g.
// image j of a group of N to rank j) fuse into one group between
// hic_gather_group_begin / _end.
//
// Reference: hiccup has no multi-GPU path; the whole-image buffers this gather
// reassembles are what codec.jpeg_encode consumes (codec.py:275-334) after the
// single-process compression.jpeg_compression (compression.py:16-39).  The
// Python side (hiccup_amd/sharding.py) does the same exchange through
// torch.distributed; this is the same transfer for a host without torch.
//
// RCCL is opened at run time (dlopen of librccl.so.1): the library loads and
// every other entry point works without it.  A process that already holds
// torch's RCCL (same soname) gets that copy, so there is one RCCL per process.
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <string.h>

#include "hic_common.h"

namespace hic {
namespace {

struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  bool ok = false;
};

const Rccl *rccl() {
  static Rccl r = [] {
    Rccl t;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return t;
#define HIC_SYM(field, name) t.field = reinterpret_cast<decltype(t.field)>(dlsym(h, name))
    HIC_SYM(get_unique_id, "ncclGetUniqueId");
    HIC_SYM(comm_init_rank, "ncclCommInitRank");
    HIC_SYM(comm_destroy, "ncclCommDestroy");
    HIC_SYM(send, "ncclSend");
    HIC_SYM(recv, "ncclRecv");
    HIC_SYM(group_start, "ncclGroupStart");
    HIC_SYM(group_end, "ncclGroupEnd");
    HIC_SYM(error_string, "ncclGetErrorString");
#undef HIC_SYM
    t.ok = t.get_unique_id && t.comm_init_rank && t.comm_destroy && t.send && t.recv && t.group_start &&
           t.group_end && t.error_string;
    return t;
  }();
  return &r;
}

int need_rccl(const Rccl *&r) {
  r = rccl();
  if (!r->ok) {
    set_error("RCCL (librccl.so.1) could not be loaded");
    return HIC_ERR_HIP;
  }
  return HIC_OK;
}

int rccl_status(const Rccl *r, ncclResult_t e, const char *what) {
  if (e != ncclSuccess) {
    set_error("%s: %s", what, r->error_string(e));
    return HIC_ERR_HIP;
  }
  return HIC_OK;
}

struct Comm {
  ncclComm_t comm;
  int world, rank;
};

}  // namespace
}  // namespace hic

using namespace hic;

extern "C" int hic_gather_unique_id(uint8_t *h_id) {
  if (!h_id) return arg_error("null pointer");
  const Rccl *r;
  if (int rc = need_rccl(r)) return rc;
  ncclUniqueId id;
  if (int rc = rccl_status(r, r->get_unique_id(&id), "ncclGetUniqueId")) return rc;
  memcpy(h_id, id.internal, HIC_GATHER_ID_BYTES);
  return HIC_OK;
}

extern "C" int hic_gather_comm_init(void **h_comm, const uint8_t *h_id, int world, int rank) {
  if (!h_comm || !h_id) return arg_error("null pointer");
  if (world < 1 || rank < 0 || rank >= world) return arg_error("rank %d of world %d", rank, world);
  *h_comm = nullptr;
  const Rccl *r;
  if (int rc = need_rccl(r)) return rc;
  ncclUniqueId id;
  memcpy(id.internal, h_id, HIC_GATHER_ID_BYTES);
  Comm *c = new Comm{nullptr, world, rank};
  if (int rc = rccl_status(r, r->comm_init_rank(&c->comm, world, id, rank), "ncclCommInitRank")) {
    delete c;
    return rc;
  }
  *h_comm = c;
  return HIC_OK;
}

extern "C" int hic_gather_comm_destroy(void *comm) {
  if (!comm) return arg_error("null communicator");
  const Rccl *r;
  if (int rc = need_rccl(r)) return rc;
  Comm *c = static_cast<Comm *>(comm);
  const int rc = rccl_status(r, r->comm_destroy(c->comm), "ncclCommDestroy");
  delete c;
  return rc;
}

extern "C" int hic_gather_group_begin(void) {
  const Rccl *r;
  if (int rc = need_rccl(r)) return rc;
  return rccl_status(r, r->group_start(), "ncclGroupStart");
}

extern "C" int hic_gather_group_end(void) {
  const Rccl *r;
  if (int rc = need_rccl(r)) return rc;
  return rccl_status(r, r->group_end(), "ncclGroupEnd");
}

extern "C" int hic_gather_bytes(void *comm, const void *d_send, int64_t send_bytes, void *d_recv,
                                const int64_t *h_recv_offsets, const int64_t *h_recv_bytes, int root, void *stream) {
  if (!comm) return arg_error("null communicator");
  Comm *c = static_cast<Comm *>(comm);
  if (root < 0 || root >= c->world) return arg_error("root %d of world %d", root, c->world);
  if (send_bytes < 0 || (send_bytes > 0 && !d_send)) return arg_error("send buffer");
  const Rccl *r;
  if (int rc = need_rccl(r)) return rc;
  const hipStream_t s = as_stream(stream);
  if (c->rank != root) {
    if (send_bytes == 0) return HIC_OK;  // the root posts no receive for an empty slice
    if (int rc = rccl_status(r, r->group_start(), "ncclGroupStart")) return rc;
    const int rc = rccl_status(r, r->send(d_send, (size_t)send_bytes, ncclUint8, root, c->comm, s), "ncclSend");
    const int rc2 = rccl_status(r, r->group_end(), "ncclGroupEnd");
    return rc ? rc : rc2;
  }
  if (!d_recv || !h_recv_offsets || !h_recv_bytes) return arg_error("root needs the receive buffer and its layout");
  for (int p = 0; p < c->world; ++p)
    if (h_recv_offsets[p] < 0 || h_recv_bytes[p] < 0) return arg_error("receive layout of rank %d", p);
  if (h_recv_bytes[root] != send_bytes) return arg_error("root's own slice: %lld bytes sent, %lld expected",
                                                         (long long)send_bytes, (long long)h_recv_bytes[root]);
  uint8_t *base = static_cast<uint8_t *>(d_recv);
  // the root's own slice: in place already, or one device copy
  if (send_bytes > 0 && base + h_recv_offsets[root] != d_send)
    if (int rc = hip_status(hipMemcpyAsync(base + h_recv_offsets[root], d_send, (size_t)send_bytes,
                                           hipMemcpyDeviceToDevice, s), "hipMemcpyAsync"))
      return rc;
  if (int rc = rccl_status(r, r->group_start(), "ncclGroupStart")) return rc;
  int rc = HIC_OK;
  for (int p = 0; p < c->world && rc == HIC_OK; ++p)
    if (p != root && h_recv_bytes[p] > 0)
      rc = rccl_status(r, r->recv(base + h_recv_offsets[p], (size_t)h_recv_bytes[p], ncclUint8, p, c->comm, s),
                       "ncclRecv");
  const int rc2 = rccl_status(r, r->group_end(), "ncclGroupEnd");
  return rc ? rc : rc2;
}

extern "C" int hic_gather_comm_info(void *comm, int *h_world, int *h_rank) {
  if (!comm || !h_world || !h_rank) return arg_error("null pointer");
  const Comm *c = static_cast<const Comm *>(comm);
  *h_world = c->world;
  *h_rank = c->rank;
  return HIC_OK;
}
