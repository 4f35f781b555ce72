// mano_comm.hip -- gather of data-parallel shards to one GPU (include/mano_hip.h
// mano_comm_* / mano_gather), RCCL over xGMI.
//
// The reference has no parallelism (mano_np.py:79-115 is one hand at a time);
// hands are independent, so the forward itself never communicates.  The only
// exchange is the optional assembly of every rank's verts / joints on one
// device (BASELINE config C4).  Its shape on MI355X: xGMI is point to point
// (7 links per GPU), so a gather is a set of direct peer -> root transfers,
// one per link, issued as one RCCL group of ncclSend / ncclRecv -- not a ring
// all-gather, whose per-hop link bandwidth would bound the whole transfer.
//
// RCCL is loaded with dlopen on first use (librccl.so.1): the forward path
// never needs it, and a process that already holds RCCL (torch) shares that
// copy because the soname matches.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/mano_hip.h"

static_assert(MANO_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");

// mano_last_error's storage lives in mano_abi.hip.
namespace mano {
int set_error(int code, const char* msg);
}

struct mano_comm {
  uint32_t magic;
  int device;
  int n_ranks;
  int rank;
  ncclComm_t comm;
};

namespace {

constexpr uint32_t kCommMagic = 0x434f4d4du;  // "COMM"

// Shards are float rows, so they move as ncclFloat: a C4 shard of 5.0 GB is
// 1.25e9 elements, inside a 32-bit count, where ncclChar would pass 5.0e9
// (RCCL takes size_t counts, but nothing larger than 2^31 elements has run
// here).  Both ends of a send / recv pair pick the type from the same byte
// count, so they always agree.
struct Elems {
  ncclDataType_t type;
  size_t count;
};
Elems elems(size_t bytes) {
  return bytes % 4 == 0 ? Elems{ncclFloat, bytes / 4} : Elems{ncclChar, bytes};
}

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return mano::set_error(code, buf);
}

struct Rccl {
  bool ok = false;
  std::string why;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* e = dlerror();
      r.why = std::string("dlopen(librccl.so.1): ") + (e ? e : "unknown error");
      return;
    }
    auto sym = [&](const char* name) {
      void* p = dlsym(h, name);
      if (!p && r.why.empty()) r.why = std::string("librccl.so.1 lacks ") + name;
      return p;
    };
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
    r.init_rank = reinterpret_cast<decltype(r.init_rank)>(sym("ncclCommInitRank"));
    r.init_all = reinterpret_cast<decltype(r.init_all)>(sym("ncclCommInitAll"));
    r.destroy = reinterpret_cast<decltype(r.destroy)>(sym("ncclCommDestroy"));
    r.send = reinterpret_cast<decltype(r.send)>(sym("ncclSend"));
    r.recv = reinterpret_cast<decltype(r.recv)>(sym("ncclRecv"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
    r.all_gather = reinterpret_cast<decltype(r.all_gather)>(sym("ncclAllGather"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
    r.ok = r.why.empty();
  });
  return r;
}

int rccl_fail(const Rccl& r, ncclResult_t res, const char* what) {
  return fail(MANO_ECOMM, "%s: %s (%d)", what, r.error_string ? r.error_string(res) : "?", int(res));
}

int check_comm(const mano_comm* c) {
  if (!c) return fail(MANO_EINVAL, "comm handle is NULL");
  if (c->magic != kCommMagic) return fail(MANO_ESTATE, "comm handle is invalid or destroyed");
  return MANO_OK;
}

struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int dev) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != dev) err = hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace

extern "C" {

int mano_comm_unique_id(unsigned char* id) {
  mano::set_error(MANO_OK, "");
  if (!id) return fail(MANO_EINVAL, "id is NULL");
  const Rccl& r = rccl();
  if (!r.ok) return fail(MANO_ECOMM, "%s", r.why.c_str());
  ncclUniqueId uid;
  ncclResult_t res = r.get_unique_id(&uid);
  if (res != ncclSuccess) return rccl_fail(r, res, "ncclGetUniqueId");
  std::memcpy(id, uid.internal, NCCL_UNIQUE_ID_BYTES);
  return MANO_OK;
}

int mano_comm_create(int device, int32_t n_ranks, int32_t rank, const unsigned char* id,
                     mano_comm** out) {
  mano::set_error(MANO_OK, "");
  if (!out) return fail(MANO_EINVAL, "out is NULL");
  *out = nullptr;
  if (!id) return fail(MANO_EINVAL, "id is NULL");
  if (device < 0) return fail(MANO_EINVAL, "device %d is negative", device);
  if (n_ranks < 1 || rank < 0 || rank >= n_ranks)
    return fail(MANO_EINVAL, "rank %d / n_ranks %d out of range", rank, n_ranks);
  const Rccl& r = rccl();
  if (!r.ok) return fail(MANO_ECOMM, "%s", r.why.c_str());
  DeviceGuard guard(device);
  if (guard.err != hipSuccess)
    return fail(MANO_EHIP, "hipSetDevice: %s", hipGetErrorString(guard.err));
  ncclUniqueId uid;
  std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t comm = nullptr;
  ncclResult_t res = r.init_rank(&comm, n_ranks, uid, rank);  // blocks until every rank joined
  if (res != ncclSuccess) return rccl_fail(r, res, "ncclCommInitRank");
  mano_comm* c = new (std::nothrow) mano_comm{kCommMagic, device, n_ranks, rank, comm};
  if (!c) {
    r.destroy(comm);
    return fail(MANO_EINVAL, "out of host memory");
  }
  *out = c;
  return MANO_OK;
}

int mano_comm_create_all(int32_t n, const int* devices, mano_comm** comms) {
  mano::set_error(MANO_OK, "");
  if (!comms) return fail(MANO_EINVAL, "comms is NULL");
  if (n < 1) return fail(MANO_EINVAL, "n %d < 1", n);
  for (int i = 0; i < n; ++i) comms[i] = nullptr;
  if (!devices) return fail(MANO_EINVAL, "devices is NULL");
  int n_dev = 0;
  hipError_t he = hipGetDeviceCount(&n_dev);
  if (he != hipSuccess) return fail(MANO_EHIP, "hipGetDeviceCount: %s", hipGetErrorString(he));
  for (int i = 0; i < n; ++i) {
    if (devices[i] < 0 || devices[i] >= n_dev)
      return fail(MANO_EINVAL, "devices[%d] = %d outside [0, %d)", i, devices[i], n_dev);
    for (int j = 0; j < i; ++j)
      if (devices[j] == devices[i])
        return fail(MANO_EINVAL, "device %d is listed twice (one communicator rank per GPU)", devices[i]);
  }
  const Rccl& r = rccl();
  if (!r.ok) return fail(MANO_ECOMM, "%s", r.why.c_str());
  std::vector<ncclComm_t> raw(n, nullptr);
  {
    DeviceGuard guard(devices[0]);  // ncclCommInitAll sets each device itself; restore the caller's
    ncclResult_t res = r.init_all(raw.data(), n, devices);  // one clique, rank i on devices[i]
    if (res != ncclSuccess) return rccl_fail(r, res, "ncclCommInitAll");
  }
  for (int i = 0; i < n; ++i) {
    comms[i] = new (std::nothrow) mano_comm{kCommMagic, devices[i], n, i, raw[i]};
    if (!comms[i]) {
      for (int j = 0; j < n; ++j) {
        if (j < i) {
          comms[j]->magic = 0;
          delete comms[j];
        }
        comms[j] = nullptr;
        r.destroy(raw[j]);
      }
      return fail(MANO_EINVAL, "out of host memory");
    }
  }
  return MANO_OK;
}

int mano_group_start(void) {
  mano::set_error(MANO_OK, "");
  const Rccl& r = rccl();
  if (!r.ok) return fail(MANO_ECOMM, "%s", r.why.c_str());
  ncclResult_t res = r.group_start();
  if (res != ncclSuccess) return rccl_fail(r, res, "ncclGroupStart");
  return MANO_OK;
}

int mano_group_end(void) {
  mano::set_error(MANO_OK, "");
  const Rccl& r = rccl();
  if (!r.ok) return fail(MANO_ECOMM, "%s", r.why.c_str());
  ncclResult_t res = r.group_end();
  if (res != ncclSuccess) return rccl_fail(r, res, "ncclGroupEnd");
  return MANO_OK;
}

int mano_comm_destroy(mano_comm* c) {
  mano::set_error(MANO_OK, "");
  if (!c) return MANO_OK;
  if (int rc = check_comm(c)) return rc;
  const Rccl& r = rccl();
  DeviceGuard guard(c->device);
  c->magic = 0;
  ncclResult_t res = r.destroy(c->comm);
  delete c;
  if (res != ncclSuccess) return rccl_fail(r, res, "ncclCommDestroy");
  return MANO_OK;
}

int mano_comm_info(const mano_comm* c, int32_t* n_ranks, int32_t* rank, int32_t* device) {
  mano::set_error(MANO_OK, "");
  if (int rc = check_comm(c)) return rc;
  if (n_ranks) *n_ranks = c->n_ranks;
  if (rank) *rank = c->rank;
  if (device) *device = c->device;
  return MANO_OK;
}

}  // extern "C"

namespace {

// Every check mano_gather makes before it touches a stream or posts an RCCL
// op; `off` (root only) receives the per-rank landing offsets.  Shared by
// mano_gather and mano_gather_check, so a call the pre-flight accepts is
// never refused by the real one.
int gather_args(const mano_comm* c, const void* send, size_t send_bytes, const void* recv,
                const size_t* rank_bytes, int32_t root, std::vector<size_t>* off) {
  if (int rc = check_comm(c)) return rc;
  if (root < 0 || root >= c->n_ranks)
    return fail(MANO_EINVAL, "root %d out of range [0, %d)", root, c->n_ranks);
  if (send_bytes > 0 && !send) return fail(MANO_EINVAL, "send is NULL");
  if (c->rank != root) return MANO_OK;
  off->assign(c->n_ranks + 1, 0);
  for (int p = 0; p < c->n_ranks; ++p) (*off)[p + 1] = (*off)[p] + (rank_bytes ? rank_bytes[p] : send_bytes);
  if (rank_bytes && rank_bytes[root] != send_bytes)
    return fail(MANO_EINVAL, "rank_bytes[root] = %zu but root sends %zu bytes", rank_bytes[root], send_bytes);
  if ((*off)[c->n_ranks] > 0 && !recv) return fail(MANO_EINVAL, "recv is NULL on root");
  return MANO_OK;
}

}  // namespace

extern "C" {

int mano_gather_check(const mano_comm* c, const void* send, size_t send_bytes, const void* recv,
                      const size_t* rank_bytes, int32_t root) {
  mano::set_error(MANO_OK, "");
  std::vector<size_t> off;
  return gather_args(c, send, send_bytes, recv, rank_bytes, root, &off);
}

int mano_gather(mano_comm* c, const void* send, size_t send_bytes, void* recv,
                const size_t* rank_bytes, int32_t root, void* stream) {
  mano::set_error(MANO_OK, "");
  std::vector<size_t> off;
  if (int rc = gather_args(c, send, send_bytes, recv, rank_bytes, root, &off)) return rc;
  const bool is_root = c->rank == root;
  const Rccl& r = rccl();
  DeviceGuard guard(c->device);
  if (guard.err != hipSuccess)
    return fail(MANO_EHIP, "hipSetDevice: %s", hipGetErrorString(guard.err));
  hipStream_t s = static_cast<hipStream_t>(stream);
  // The root's own shard: copied into place, unless the caller computed it
  // there (send == its slot of recv: nothing to move).
  if (is_root && send_bytes > 0 && send != static_cast<const char*>(recv) + off[root]) {
    hipError_t e = hipMemcpyAsync(static_cast<char*>(recv) + off[root], send, send_bytes,
                                  hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return fail(MANO_EHIP, "hipMemcpyAsync: %s", hipGetErrorString(e));
  }
  if (c->n_ranks == 1) return MANO_OK;
  ncclResult_t res = r.group_start();
  if (res != ncclSuccess) return rccl_fail(r, res, "ncclGroupStart");
  if (is_root) {
    for (int p = 0; p < c->n_ranks && res == ncclSuccess; ++p) {
      const size_t b = off[p + 1] - off[p];
      if (p != root && b > 0) {
        const Elems e = elems(b);
        res = r.recv(static_cast<char*>(recv) + off[p], e.count, e.type, p, c->comm, s);
      }
    }
  } else if (send_bytes > 0) {
    const Elems e = elems(send_bytes);
    res = r.send(send, e.count, e.type, root, c->comm, s);
  }
  const ncclResult_t end = r.group_end();
  if (res != ncclSuccess) return rccl_fail(r, res, is_root ? "ncclRecv" : "ncclSend");
  if (end != ncclSuccess) return rccl_fail(r, end, "ncclGroupEnd");
  return MANO_OK;
}

int mano_allgather(mano_comm* c, const void* send, size_t send_bytes, void* recv, void* stream) {
  mano::set_error(MANO_OK, "");
  if (int rc = check_comm(c)) return rc;
  if (send_bytes == 0) return MANO_OK;
  if (!send) return fail(MANO_EINVAL, "send is NULL");
  if (!recv) return fail(MANO_EINVAL, "recv is NULL");
  const Rccl& r = rccl();
  DeviceGuard guard(c->device);
  if (guard.err != hipSuccess)
    return fail(MANO_EHIP, "hipSetDevice: %s", hipGetErrorString(guard.err));
  // RCCL's ring all-gather: each of the n - 1 steps forwards one shard to the
  // next rank, so every shard crosses n - 1 links in turn.
  const Elems e = elems(send_bytes);
  ncclResult_t res = r.all_gather(send, recv, e.count, e.type, c->comm, static_cast<hipStream_t>(stream));
  if (res != ncclSuccess) return rccl_fail(r, res, "ncclAllGather");
  return MANO_OK;
}

}  // extern "C"
