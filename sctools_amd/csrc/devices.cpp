// Several GPUs from one process (SURVEY §8(b) `n_gpus`, §8(e)): the library's own device split,
// so a drop-in caller on an 8-GPU node -- Barcodes.summarize_hamming_distances, nearest-whitelist
// correction, the host encode stream -- uses every GPU without torch.distributed.
//
// A slot is one (worker thread, device) pair: slot r of a call runs on persistent worker thread r
// with devices[r] current, so the thread-local host stages, pinned buffers and pipeline streams of
// the *_host entry points are created once per slot and reused.  Repeated devices are logical
// shards of one GPU (the tests run [0, 0] and [0, 0, 0, 0] on a one-GPU box).
//
// The split follows SURVEY §8(e): all-pairs -> contiguous item (transform slice) ranges, each
// device with its own replica of the codes, and the small counts vectors summed on the host --
// they have to come back to the host anyway, so a device collective would only add a hop;
// nearest and the encode stream -> contiguous record ranges, no exchange at all.
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "sct_common.h"

namespace sct {
namespace {

struct WorkerPool {
  std::mutex call_mu;  // one multi-device call at a time
  std::mutex mu;
  std::condition_variable go, done;
  uint64_t gen = 0;
  int active = 0, pending = 0, nthreads = 0;
  const int* devices = nullptr;
  const std::function<int(int)>* fn = nullptr;
  std::vector<int> rc;
  std::vector<std::string> err;

  void loop(int r) {
    uint64_t seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> lk(mu);
      go.wait(lk, [&] { return gen != seen; });
      seen = gen;
      if (r >= active) continue;  // (not part of this call)
      const std::function<int(int)>* f = fn;
      const int dev = devices[r];
      lk.unlock();
      int c = SCT_OK;
      const hipError_t e = hipSetDevice(dev);
      if (e != hipSuccess)
        c = fail(SCT_E_HIP, "hipSetDevice(%d): %s", dev, hipGetErrorString(e));
      else
        c = (*f)(r);
      std::string msg = c != SCT_OK ? std::string(last_error()) : std::string();
      lk.lock();
      rc[(size_t)r] = c;
      err[(size_t)r] = std::move(msg);
      if (--pending == 0) done.notify_all();
    }
  }
};

// never destroyed: its threads wait on it until the process exits
WorkerPool* workers() {
  static WorkerPool* p = new WorkerPool();
  return p;
}

}  // namespace

int run_on_devices(const int* devices, int ndev, const std::function<int(int)>& fn) {
  if (!devices || ndev <= 1) {
    if (!devices || ndev < 1) return fn(0);
    int cur = 0;
    SCT_HIP(hipGetDevice(&cur));
    if (cur == devices[0]) return fn(0);
    SCT_HIP(hipSetDevice(devices[0]));
    const int rc = fn(0);
    (void)hipSetDevice(cur);
    return rc;
  }
  int count = 0;
  SCT_HIP(hipGetDeviceCount(&count));
  for (int r = 0; r < ndev; ++r)
    if (devices[r] < 0 || devices[r] >= count)
      return fail(SCT_E_INVALID, "device %d of slot %d: %d devices visible", devices[r], r, count);
  SCT_CHECK(ndev <= 64, "at most 64 device slots (got %d)", ndev);
  WorkerPool* p = workers();
  std::lock_guard<std::mutex> call(p->call_mu);
  {
    std::lock_guard<std::mutex> lk(p->mu);
    while (p->nthreads < ndev) {
      const int r = p->nthreads++;
      std::thread([p, r] { p->loop(r); }).detach();
    }
    p->rc.assign((size_t)ndev, SCT_OK);
    p->err.assign((size_t)ndev, std::string());
    p->devices = devices;
    p->fn = &fn;
    p->active = ndev;
    p->pending = ndev;
    ++p->gen;
  }
  p->go.notify_all();
  std::unique_lock<std::mutex> lk(p->mu);
  p->done.wait(lk, [&] { return p->pending == 0; });
  for (int r = 0; r < ndev; ++r)
    if (p->rc[(size_t)r] != SCT_OK) return fail(p->rc[(size_t)r], "device slot %d (device %d): %s", r, devices[r],
                                                p->err[(size_t)r].c_str());
  return SCT_OK;
}

}  // namespace sct

namespace {
inline int64_t split(int64_t n, int r, int k) { return n * r / k; }
}  // namespace

extern "C" int sct_nearest_host_devices(int kind, const uint64_t* whitelist, int64_t nw, const uint64_t* queries,
                                        int64_t nq, int code_bits, int max_d, const int* devices, int ndev,
                                        int32_t* index, uint8_t* dist) {
  SCT_CHECK(nw >= 0 && nq >= 0, "bad sizes");
  const int k = std::max(ndev, 1);
  return sct::run_on_devices(devices, ndev, [&](int r) {
    const int64_t b = split(nq, r, k), e = split(nq, r + 1, k);
    return sct_nearest_host(kind, whitelist, nw, queries + b, e - b, code_bits, max_d, index + b, dist + b);
  });
}

// a whitelist index on every slot's device (the whitelist is replicated: 5.9 MB at 737K)
struct sct_nearest_multi {
  std::vector<int> devices;
  std::vector<sct_nearest_plan*> plans;
};

extern "C" int sct_nearest_multi_create_host(int kind, const uint64_t* whitelist, int64_t nw, int code_bits, int max_d,
                                             const int* devices, int ndev, sct_nearest_multi** out) {
  SCT_CHECK(out != nullptr, "plan is NULL");
  SCT_CHECK(ndev >= 1 && devices != nullptr, "need at least one device");
  *out = nullptr;
  auto* m = new sct_nearest_multi();
  m->devices.assign(devices, devices + ndev);
  m->plans.assign((size_t)ndev, nullptr);
  const int rc = sct::run_on_devices(m->devices.data(), ndev, [&](int r) {
    return sct_nearest_plan_create_host(kind, whitelist, nw, code_bits, max_d, &m->plans[(size_t)r]);
  });
  if (rc != SCT_OK) {
    sct_nearest_multi_destroy(m);
    return rc;
  }
  *out = m;
  return SCT_OK;
}

extern "C" int sct_nearest_multi_query_host(sct_nearest_multi* m, const uint64_t* queries, int64_t nq, int32_t* index,
                                            uint8_t* dist) {
  SCT_CHECK(m != nullptr, "plan is NULL");
  SCT_CHECK(nq >= 0 && (nq == 0 || (queries && index && dist)), "bad arguments");
  if (nq == 0) return SCT_OK;
  const int k = (int)m->plans.size();
  return sct::run_on_devices(m->devices.data(), k, [&](int r) {
    const int64_t b = split(nq, r, k), e = split(nq, r + 1, k);
    return sct_nearest_query_host(m->plans[(size_t)r], queries + b, e - b, index + b, dist + b);
  });
}

extern "C" int sct_nearest_multi_destroy(sct_nearest_multi* m) {
  if (!m) return SCT_OK;
  // each index freed on its own slot (its device current), after the work it enqueued
  (void)sct::run_on_devices(m->devices.data(), (int)m->plans.size(), [&](int r) {
    return m->plans[(size_t)r] ? sct_nearest_plan_destroy(m->plans[(size_t)r]) : SCT_OK;
  });
  delete m;
  return SCT_OK;
}

extern "C" int sct_encode_stream_host_devices(int kind, const uint8_t* seqs, int64_t n, int L, uint64_t* codes,
                                              uint8_t* gc, uint8_t* flags, int64_t chunk, const int* devices,
                                              int ndev) {
  SCT_CHECK(n >= 0 && L >= 1, "bad sizes");
  const int k = std::max(ndev, 1);
  return sct::run_on_devices(devices, ndev, [&](int r) {
    const int64_t b = split(n, r, k), e = split(n, r + 1, k);
    if (e == b) return SCT_OK;
    return sct_encode_stream_host(kind, seqs + b * L, e - b, L, codes + b, gc + b, flags + b, chunk);
  });
}
