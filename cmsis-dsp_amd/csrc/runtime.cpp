// Host runtime: device table cache, staging scratch, error channel.
#include "runtime.hpp"

#include "kernels.hpp"

#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <link.h>
#include <string.h>

#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/arm_math_mi355x.h"

#ifndef MI355X_SYNC_DEFAULT
#define MI355X_SYNC_DEFAULT 1
#endif

namespace mi355x {

namespace {
thread_local int g_err = 0;
thread_local std::string g_err_msg;

std::mutex g_table_mu;
std::map<std::tuple<int, const void*, size_t>, void*> g_tables;
// library-address bit-reversal tables: their verdict and, when not canonical, the permutation
// (re-resolved through the blob cache on every call: no raw blob pointer is kept here)
struct PermEntry { bool canon = true; std::vector<uint16_t> perm; };
std::map<std::tuple<int, const void*, uint16_t, int, int>, PermEntry> g_perms;

// ---- content-keyed blob cache --------------------------------------------------------------
// An LRU bounded in bytes PER DEVICE (default 256 MiB, arm_mi355x_set_table_cache_limit).
// Lifetime rules (round 4):
//  * a blob handed out inside a BlobScope is HELD (holds > 0) until the scope ends, so no other
//    thread's insertion -- and no later lookup of the same call -- can evict it before the
//    launches that read it are enqueued;
//  * the scope then records one event on its stream after that work; the blob keeps the events
//    of its uses that may still be pending;
//  * eviction never synchronizes the device and never runs under g_table_mu: the victim leaves
//    the map under the lock, and afterwards its memory is released with hipFreeAsync on a
//    per-device reclaim stream made to wait on the victim's use events (stream order, so later
//    work on other streams is not stalled).
// Blobs are allocated with hipMallocAsync (stream-ordered pool) on a per-device upload stream.
// All state lives in heap objects that are never destroyed: no static-destruction ordering.
struct EvPool {
  std::mutex mu;
  std::map<int, std::vector<hipEvent_t>> free;
};
EvPool& ev_pool() { static EvPool* p = new EvPool; return *p; }

struct Ev {                       // one recorded use event, shared by the blobs of one scope
  hipEvent_t e = nullptr;
  int d = 0;
  ~Ev() {
    if (!e) return;
    EvPool& p = ev_pool();
    std::lock_guard<std::mutex> lk(p.mu);
    p.free[d].push_back(e);
  }
};
using EvRef = std::shared_ptr<Ev>;

struct Blob {
  std::vector<uint8_t> host;
  void* dev = nullptr;
  int d = 0;
  uint64_t tick = 0;
  int holds = 0;                  // live BlobScopes holding it
  bool unscoped = false;          // handed out with no scope: released after a device sync
  std::vector<EvRef> uses;        // events after the enqueued work that reads it
};
using BlobRef = std::shared_ptr<Blob>;

struct BlobCache {
  std::map<std::tuple<int, uint64_t, size_t>, std::vector<BlobRef>> map;
  std::map<int, size_t> bytes;    // per device
  size_t limit = size_t(256) << 20;
  uint64_t tick = 0;
};
BlobCache& cache() { static BlobCache* c = new BlobCache; return *c; }   // under g_table_mu

thread_local std::vector<BlobRef> t_held;   // blobs held by this thread's live scopes
thread_local int t_scopes = 0;

// per-device internal streams of the cache (created once, never destroyed)
std::mutex g_cache_stream_mu;
hipStream_t cache_stream(int d, int which) {
  static std::map<std::pair<int, int>, hipStream_t>* m = new std::map<std::pair<int, int>, hipStream_t>;
  std::lock_guard<std::mutex> lk(g_cache_stream_mu);
  auto it = m->find({d, which});
  if (it != m->end()) return it->second;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  (*m)[{d, which}] = s;
  return s;
}
enum { kUploadStream = 0, kReclaimStream = 1 };

// drop events whose work has completed (caller holds g_table_mu)
void prune_uses(Blob& b) {
  b.uses.erase(std::remove_if(b.uses.begin(), b.uses.end(),
                              [](const EvRef& r) { return hipEventQuery(r->e) == hipSuccess; }),
               b.uses.end());
}

// take least-recently-used, unheld blobs of device d out of the map until `incoming` more bytes
// fit (caller holds g_table_mu); returns them for release_blobs() outside the lock
std::vector<BlobRef> evict_locked(int d, size_t incoming) {
  BlobCache& c = cache();
  std::vector<BlobRef> out;
  size_t& used = c.bytes[d];
  while (used + incoming > c.limit && used > 0) {
    auto vb = c.map.end();
    size_t vi = 0;
    uint64_t oldest = UINT64_MAX;
    for (auto it = c.map.begin(); it != c.map.end(); ++it) {
      if (std::get<0>(it->first) != d) continue;
      for (size_t i = 0; i < it->second.size(); ++i) {
        const Blob& b = *it->second[i];
        if (b.holds == 0 && b.tick < oldest) { oldest = b.tick; vb = it; vi = i; }
      }
    }
    if (vb == c.map.end()) break;             // everything left is held by a live call
    BlobRef v = vb->second[vi];
    used -= v->host.size();
    vb->second.erase(vb->second.begin() + (long)vi);
    if (vb->second.empty()) c.map.erase(vb);
    out.push_back(std::move(v));
  }
  return out;
}

// release evicted blobs (no lock held): stream-ordered after every recorded use
void release_blobs(std::vector<BlobRef>& victims) {
  if (victims.empty()) return;
  int prev = 0;
  (void)hipGetDevice(&prev);
  for (BlobRef& v : victims) {
    if (v->d != prev) (void)hipSetDevice(v->d);
    hipStream_t rs = cache_stream(v->d, kReclaimStream);
    if (v->unscoped || !rs) (void)hipDeviceSynchronize();   // a use the cache could not track
    else
      for (const EvRef& r : v->uses) (void)hipStreamWaitEvent(rs, r->e, 0);
    (void)hipFreeAsync(v->dev, rs);
    v->uses.clear();
    if (v->d != prev) (void)hipSetDevice(prev);
  }
  victims.clear();
}

// hand out blob b (caller holds g_table_mu): held by the innermost scope, if any.  Every entry
// point declares a BlobScope before its first table fetch; a hand-out without one marks the blob
// `unscoped` for good (its eviction then synchronizes the device, the one way to know an untracked
// use has finished).  Builds with -DMI355X_DEBUG_SCOPES abort on such a hand-out instead, so a
// future entry point that forgets its scope is caught in testing.
const void* hand_out(const BlobRef& b) {
  b->tick = ++cache().tick;
  if (t_scopes > 0) {
    ++b->holds;
    t_held.push_back(b);
  } else {
#ifdef MI355X_DEBUG_SCOPES
    fprintf(stderr, "cmsisdsp-mi355x: table handed out outside a BlobScope\n");
    abort();
#endif
    b->unscoped = true;
  }
  return b->dev;
}

uint64_t fnv1a(const uint8_t* p, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ull; }
  return h;
}

int cur_dev() { int d = 0; (void)hipGetDevice(&d); return d; }

// ---- per-thread resources of the synchronous drop-in path ----------------------------------
// The reference allocates nothing (SURVEY §8b "Ownership"); this backend needs, per calling
// thread, a non-blocking stream per device, device scratch, pinned and coherent-pinned staging
// and a coherent completion word.  They are owned by ONE thread_local object, so a thread that
// exits gives them back: its destructor drains and destroys the streams, then frees the scratch,
// the staging and the completion words.  The process's main thread keeps the
// deliberate leak at process exit -- its thread_local destructors run during static destruction,
// when the HIP runtime may already be gone.  arm_mi355x_release_thread_resources() releases the
// calling thread's set explicitly (thread pools that recycle threads; the main thread).
struct Scratch { void* p = nullptr; size_t n = 0; };
struct Pinned { void* p = nullptr; size_t n = 0; };
struct DoneWord { volatile uint32_t* h = nullptr; uint32_t* d = nullptr; uint32_t seq = 0; };

std::atomic<int> g_live_owners{0};     // threads currently holding any of the resources below

bool is_main_thread() { return (pid_t)syscall(SYS_gettid) == getpid(); }

struct ThreadRes {
  std::map<std::pair<int, int>, Scratch> scratch;   // (device, slot)
  std::map<int, Pinned> pinned;                     // slot
  std::map<int, Pinned> zpinned;                    // slot; coherent, device-accessed in place
  std::map<int, hipStream_t> streams;               // device
  std::map<int, DoneWord> done;                     // device
  bool counted = false;

  void touch() {
    if (!counted) { counted = true; g_live_owners.fetch_add(1, std::memory_order_relaxed); }
  }
  void release() {
    int prev = 0;
    const bool have_prev = hipGetDevice(&prev) == hipSuccess;
    for (auto& kv : streams) {                      // nothing of this thread may still be in flight
      (void)hipSetDevice(kv.first);
      (void)hipStreamSynchronize(kv.second);
      (void)hipStreamDestroy(kv.second);
    }
    streams.clear();
    for (auto& kv : scratch) {
      if (!kv.second.p) continue;
      (void)hipSetDevice(kv.first.first);
      (void)hipFree(kv.second.p);
    }
    scratch.clear();
    for (auto& kv : pinned) if (kv.second.p) (void)hipHostFree(kv.second.p);
    pinned.clear();
    for (auto& kv : zpinned) if (kv.second.p) (void)hipHostFree(kv.second.p);
    zpinned.clear();
    for (auto& kv : done) if (kv.second.h) (void)hipHostFree((void*)kv.second.h);
    done.clear();
    if (have_prev) (void)hipSetDevice(prev);
    (void)hipGetLastError();
    if (counted) { counted = false; g_live_owners.fetch_sub(1, std::memory_order_relaxed); }
  }
  ~ThreadRes() {
    if (counted && !is_main_thread()) release();
  }
};
thread_local ThreadRes t_res;

// canonical permutations the reference tables induce (verified in tests/test_tables.py):
// f32: position holding frequency k under the mixed-radix [FIRST, 8, 8, ...] DIF
int f32_src(int n, int k) {
  int first = (n == 16 || n == 128 || n == 1024) ? 2 : (n == 32 || n == 256 || n == 2048) ? 4 : 1;
  int p = 0, rem = n;
  if (first > 1) { rem /= first; p += (k % first) * rem; k /= first; }
  while (rem > 1) { rem >>= 3; p += (k & 7) * rem; k >>= 3; }
  return p;
}
int fixed_src(int n, int k) {
  int bits = 0;
  while ((1 << bits) < n) ++bits;
  int r = 0;
  for (int b = 0; b < bits; ++b) r |= ((k >> b) & 1) << (bits - 1 - b);
  return r;
}
}  // namespace

void set_error(hipError_t e, const char* where) {
  g_err = (int)e;
  g_err_msg = std::string(where) + ": " + hipGetErrorString(e);
}
void clear_error() { g_err = 0; g_err_msg.clear(); }

bool is_device_ptr(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  hipError_t e = hipPointerGetAttributes(&a, p);
  if (e != hipSuccess) { (void)hipGetLastError(); return false; }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

// The address range of this library's loaded segments, found once (dl_iterate_phdr), so the
// per-call test is two compares instead of a dladdr symbol lookup.
namespace {
struct AddrRange { uintptr_t lo = 0, hi = 0; };
int find_self(dl_phdr_info* info, size_t, void* data) {
  auto* r = static_cast<AddrRange*>(data);
  const uintptr_t fn = (uintptr_t)&find_self;
  uintptr_t lo = UINTPTR_MAX, hi = 0;
  bool mine = false;
  for (int i = 0; i < info->dlpi_phnum; ++i) {
    const ElfW(Phdr)& ph = info->dlpi_phdr[i];
    if (ph.p_type != PT_LOAD) continue;
    const uintptr_t a = info->dlpi_addr + ph.p_vaddr, b = a + ph.p_memsz;
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
    mine |= fn >= a && fn < b;
  }
  if (!mine) return 0;
  r->lo = lo;
  r->hi = hi;
  return 1;
}
const AddrRange& self_range() {
  static const AddrRange r = [] {
    AddrRange x;
    dl_iterate_phdr(find_self, &x);
    return x;
  }();
  return r;
}
}  // namespace

bool is_library_addr(const void* p) {
  const AddrRange& r = self_range();
  return p && (uintptr_t)p >= r.lo && (uintptr_t)p < r.hi;
}

const void* device_table(const void* host, size_t bytes) {
  if (!host || !bytes) { set_error(hipErrorInvalidValue, "device_table: null table"); return nullptr; }
  // the library's own CommonTables first: no pointer-attribute query on the drop-in's hot path
  if (!is_library_addr(host)) return is_device_ptr(host) ? host : device_blob(host, bytes);
  const int dev = cur_dev();
  std::lock_guard<std::mutex> lk(g_table_mu);
  auto key = std::make_tuple(dev, host, bytes);
  auto it = g_tables.find(key);
  if (it != g_tables.end()) return it->second;
  void* d = nullptr;
  hipError_t e = hipMalloc(&d, bytes);
  if (e != hipSuccess) { set_error(e, "device_table: hipMalloc"); return nullptr; }
  e = hipMemcpy(d, host, bytes, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    set_error(e, "device_table: hipMemcpy");
    (void)hipFree(d);
    return nullptr;
  }
  g_tables[key] = d;
  return d;
}

const void* device_blob(const void* host, size_t bytes) {
  if (!host || !bytes) { set_error(hipErrorInvalidValue, "device_blob: empty"); return nullptr; }
  const uint8_t* h = (const uint8_t*)host;
  const int dev = cur_dev();
  const auto key = std::make_tuple(dev, fnv1a(h, bytes), bytes);
  std::vector<BlobRef> victims;
  {
    std::lock_guard<std::mutex> lk(g_table_mu);
    auto it = cache().map.find(key);
    if (it != cache().map.end())
      for (const BlobRef& b : it->second)
        if (memcmp(b->host.data(), h, bytes) == 0) return hand_out(b);
    victims = evict_locked(dev, bytes);
  }
  release_blobs(victims);
  auto b = std::make_shared<Blob>();
  b->host.assign(h, h + bytes);
  b->d = dev;
  hipStream_t us = cache_stream(dev, kUploadStream);
  if (!us) { set_error(hipErrorOutOfMemory, "device_blob: stream"); return nullptr; }
  hipError_t e = hipMallocAsync(&b->dev, bytes, us);
  if (e != hipSuccess) { set_error(e, "device_blob: hipMallocAsync"); return nullptr; }
  e = hipMemcpyAsync(b->dev, b->host.data(), bytes, hipMemcpyHostToDevice, us);
  if (e == hipSuccess) e = hipStreamSynchronize(us);
  if (e != hipSuccess) {
    set_error(e, "device_blob: upload");
    (void)hipFreeAsync(b->dev, us);
    return nullptr;
  }
  std::lock_guard<std::mutex> lk(g_table_mu);
  cache().map[key].push_back(b);
  cache().bytes[dev] += bytes;
  return hand_out(b);
}

const void* device_split_records(const void* A, const void* B, uint32_t mod, uint32_t L, int elem, hipStream_t st,
                                 bool* symmetric) {
  if (symmetric) *symmetric = false;
  if (!A || !B || !mod || !L || (elem != 2 && elem != 4)) {
    set_error(hipErrorInvalidValue, "split records");
    return nullptr;
  }
  const int dev = cur_dev();
  const bool lib = is_library_addr(A) && is_library_addr(B);
  using Key = std::tuple<int, const void*, const void*, uint32_t, uint32_t, int>;
  struct Built { void* d; bool sym; };
  static std::map<Key, Built>* built = new std::map<Key, Built>;   // library tables: never freed
  const Key key{dev, A, B, mod, L, elem};
  if (lib) {
    std::lock_guard<std::mutex> lk(g_table_mu);
    auto it = built->find(key);
    if (it != built->end()) {
      if (symmetric) *symmetric = it->second.sym;
      return it->second.d;
    }
  }
  // the words read: A/B[2 mod k + {0, 1}] for k < L
  const size_t words = 2 * (size_t)mod * (L - 1) + 2, wb = words * (size_t)elem;
  std::vector<uint8_t> ha(wb), hb(wb);
  for (int s = 0; s < 2; ++s) {
    const void* src = s ? B : A;
    uint8_t* dst = s ? hb.data() : ha.data();
    if (is_device_ptr(src)) {
      // on the call's stream: ordered after whatever the caller enqueued there (e.g. the table's
      // own upload on a non-blocking stream), which a null-stream copy is not
      if (hipMemcpyAsync(dst, src, wb, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
        set_error(hipErrorInvalidValue, "split records: table copy");
        return nullptr;
      }
    } else {
      memcpy(dst, src, wb);
    }
  }
  std::vector<uint8_t> rec((size_t)L * 4 * elem);
  for (uint32_t k = 0; k < L; ++k) {
    const size_t c = 2 * (size_t)mod * k * elem;
    uint8_t* r = rec.data() + (size_t)k * 4 * elem;
    memcpy(r, ha.data() + c, 2 * (size_t)elem);
    memcpy(r + 2 * elem, hb.data() + c, 2 * (size_t)elem);
  }
  const size_t rb = rec.size();
  // record L - k = record k with A1, B1 negated (mod 2^32 / 2^16), for every k in 1 .. L - 1: the
  // fused N = 8192 q31 inverse then stages records 0 .. L/2 only
  bool sym = true;
  for (uint32_t k = 1; k < L && sym; ++k) {
    const uint8_t* r1 = rec.data() + (size_t)k * 4 * elem;
    const uint8_t* r2 = rec.data() + (size_t)(L - k) * 4 * elem;
    for (int w = 0; w < 4 && sym; ++w) {
      int64_t x = 0, y = 0;
      if (elem == 4) { int32_t a, b; memcpy(&a, r1 + 4 * w, 4); memcpy(&b, r2 + 4 * w, 4); x = a; y = b; }
      else { int16_t a, b; memcpy(&a, r1 + 2 * w, 2); memcpy(&b, r2 + 2 * w, 2); x = a; y = b; }
      const int64_t m = elem == 4 ? (int64_t(1) << 32) : (int64_t(1) << 16);
      const int64_t want = (w & 1) ? ((-x) % m + m) % m : (x % m + m) % m;
      sym = ((y % m + m) % m) == want;
    }
  }
  if (symmetric) *symmetric = sym;
  if (!lib) return device_blob(rec.data(), rb);
  void* d = nullptr;
  hipError_t e = hipMalloc(&d, rb);
  if (e == hipSuccess) e = hipMemcpy(d, rec.data(), rb, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    set_error(e, "split records: upload");
    if (d) (void)hipFree(d);
    return nullptr;
  }
  std::lock_guard<std::mutex> lk(g_table_mu);
  auto ins = built->emplace(key, Built{d, sym});
  if (!ins.second) { (void)hipFree(d); return ins.first->second.d; }   // another thread built it first
  return d;
}

size_t blob_cache_bytes() {
  std::lock_guard<std::mutex> lk(g_table_mu);
  size_t s = 0;
  for (const auto& kv : cache().bytes) s += kv.second;
  return s;
}
void set_blob_cache_limit(size_t bytes) {
  std::vector<BlobRef> victims;
  {
    std::lock_guard<std::mutex> lk(g_table_mu);
    cache().limit = bytes;
    std::vector<int> devs;
    for (const auto& kv : cache().bytes) devs.push_back(kv.first);
    for (int d : devs) {
      std::vector<BlobRef> v = evict_locked(d, 0);
      victims.insert(victims.end(), v.begin(), v.end());
    }
  }
  release_blobs(victims);
}

BlobScope::BlobScope(hipStream_t st) : st_(st), base_(t_held.size()), dev_(cur_dev()) { ++t_scopes; }

BlobScope::~BlobScope() {
  --t_scopes;
  if (t_held.size() <= base_) return;
  // Insertions made while every other blob was held may have left the cache over its limit
  // (held blobs are never evicted); the scope that drops the last hold trims it back, so the
  // limit holds again whenever no call is live.
  std::vector<BlobRef> victims;
  if (synced_) {                            // nothing of this call is still pending
    {
      std::lock_guard<std::mutex> lk(g_table_mu);
      for (size_t i = base_; i < t_held.size(); ++i) --t_held[i]->holds;
      if (cache().bytes[dev_] > cache().limit) victims = evict_locked(dev_, 0);
    }
    t_held.resize(base_);
    release_blobs(victims);
    return;
  }
  // one event after everything this scope enqueued on st_, attached to every blob it held
  EvRef ev;
  {
    hipEvent_t e = nullptr;
    {
      EvPool& p = ev_pool();
      std::lock_guard<std::mutex> lk(p.mu);
      auto& f = p.free[dev_];
      if (!f.empty()) { e = f.back(); f.pop_back(); }
    }
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != dev_) (void)hipSetDevice(dev_);
    if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
    if (e && hipEventRecord(e, st_) == hipSuccess) {
      ev = std::make_shared<Ev>();
      ev->e = e;
      ev->d = dev_;
    } else if (e) {
      (void)hipEventDestroy(e);
    }
    if (prev != dev_) (void)hipSetDevice(prev);
  }
  {
    std::lock_guard<std::mutex> lk(g_table_mu);
    for (size_t i = base_; i < t_held.size(); ++i) {
      Blob& b = *t_held[i];
      prune_uses(b);
      if (ev) b.uses.push_back(ev);
      else b.unscoped = true;                // untracked use: release after a device sync
      --b.holds;
    }
    if (cache().bytes[dev_] > cache().limit) victims = evict_locked(dev_, 0);
  }
  t_held.resize(base_);
  release_blobs(victims);
}

const uint16_t* device_perm(int n, const uint16_t* table, uint16_t len, int kind, bool* canonical, bool* ok) {
  *ok = true;
  *canonical = true;
  if (!table) { return nullptr; }
  const int dev = cur_dev();
  // the library's own tables are immutable: cache their verdict (and permutation) by address;
  // any other table is re-derived from its current words on every call (O(len)).  A
  // non-canonical permutation is always resolved through the content-keyed blob cache.
  const bool lib = is_library_addr(table);
  auto key = std::make_tuple(dev, (const void*)table, len, kind, n);
  std::vector<uint16_t> a;
  bool canon = true, cached = false;
  if (lib) {
    std::lock_guard<std::mutex> lk(g_table_mu);
    auto it = g_perms.find(key);
    if (it != g_perms.end()) {
      canon = it->second.canon;
      if (!canon) a = it->second.perm;
      cached = true;
    }
  }
  if (!cached) {
    // apply the reference's sequential swaps (arm_bitreversal2.c:84-108) to an identity
    // array of complex indices: a[pos] = pre-reversal index that ends up at pos.
    const uint16_t* host = table;
    std::vector<uint16_t> tmp;
    if (is_device_ptr(table)) {
      tmp.resize(len);
      if (hipMemcpy(tmp.data(), table, len * sizeof(uint16_t), hipMemcpyDeviceToHost) != hipSuccess) { *ok = false; return nullptr; }
      host = tmp.data();
    }
    a.resize(n);
    for (int i = 0; i < n; ++i) a[i] = (uint16_t)i;
    for (int i = 0; i + 1 < len; i += 2) {
      const int x = host[i] >> 3, y = host[i + 1] >> 3;
      if (x >= n || y >= n) { *ok = false; return nullptr; }
      std::swap(a[x], a[y]);
    }
    for (int k = 0; k < n && canon; ++k) canon = a[k] == (kind == 0 ? f32_src(n, k) : fixed_src(n, k));
    if (lib) {
      std::lock_guard<std::mutex> lk(g_table_mu);
      PermEntry& pe = g_perms[key];
      pe.canon = canon;
      if (!canon) pe.perm = a;
    }
  }
  *canonical = canon;
  if (canon) return nullptr;
  const void* d = device_blob(a.data(), n * sizeof(uint16_t));
  if (!d) { *ok = false; return nullptr; }
  return (const uint16_t*)d;
}

void* scratch(size_t bytes, int slot) {
  const int dev = cur_dev();
  t_res.touch();
  Scratch& s = t_res.scratch[{dev, slot}];
  if (s.n < bytes) {
    if (s.p) (void)hipFree(s.p);
    s.p = nullptr;
    s.n = 0;
    if (hipMalloc(&s.p, bytes) != hipSuccess) return nullptr;
    s.n = bytes;
  }
  return s.p;
}

void* pinned(size_t bytes, int slot) {
  t_res.touch();
  Pinned& s = t_res.pinned[slot];
  if (s.n < bytes) {
    if (s.p) (void)hipHostFree(s.p);
    s.p = nullptr;
    s.n = 0;
    if (hipHostMalloc(&s.p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    s.n = bytes;
  }
  return s.p;
}

static void* zpinned(size_t bytes, int slot) {
  t_res.touch();
  Pinned& s = t_res.zpinned[slot];
  if (s.n < bytes) {
    if (s.p) (void)hipHostFree(s.p);
    s.p = nullptr;
    s.n = 0;
    if (hipHostMalloc(&s.p, bytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return nullptr;
    s.n = bytes;
  }
  return s.p;
}

void* HostIO::zin(const void* host, size_t bytes) {
  void* z = zpinned(bytes ? bytes : 4, zslot_++);
  if (z && bytes) memcpy(z, host, bytes);
  return z;
}

void* HostIO::zout(void* host, size_t bytes) {
  if (nouts_ == 6) return nullptr;
  void* z = zpinned(bytes ? bytes : 4, zslot_++);
  if (z && bytes) outs_[nouts_++] = {host, z, bytes};
  return z;
}

void* HostIO::zinout(void* host, size_t bytes) {
  if (nouts_ == 6) return nullptr;
  void* z = zin(host, bytes);
  if (z && bytes) outs_[nouts_++] = {host, z, bytes};
  return z;
}

hipError_t HostIO::in(void* dev, const void* host, size_t bytes) {
  if (!bytes) return hipSuccess;
  void* pin = pinned(bytes, slot_++);
  if (!pin) return hipErrorOutOfMemory;
  memcpy(pin, host, bytes);
  return hipMemcpyAsync(dev, pin, bytes, hipMemcpyHostToDevice, st_);
}

hipError_t HostIO::out(void* host, const void* dev, size_t bytes) {
  if (!bytes) return hipSuccess;
  if (nouts_ == 6) return hipErrorInvalidValue;
  void* pin = pinned(bytes, slot_++);
  if (!pin) return hipErrorOutOfMemory;
  hipError_t e = hipMemcpyAsync(pin, dev, bytes, hipMemcpyDeviceToHost, st_);
  if (e == hipSuccess) outs_[nouts_++] = {host, pin, bytes};
  return e;
}

// A call that returns early after queueing a copy must not leave a DMA reading a pinned slot
// that the next call overwrites (or frees, when it needs a larger one): drain the stream.
HostIO::~HostIO() {
  if ((slot_ > 0 || zslot_ > 0) && !finished_) (void)hipStreamSynchronize(st_);
}

// Completion of a synchronous drop-in call.  Spin mode (default): a one-lane
// kernel after the call's work stores a per-thread sequence number into a coherent,
// device-mapped host word (sync.hip), and the host spins on that word (bounded; then
// hipStreamSynchronize, which also reports errors) instead of the runtime's blocking wait.
// CMSISDSP_MI355X_SYNC=sync|spin overrides the default (MI355X_SYNC_DEFAULT).
namespace {
int sync_mode() {
  static const int m = [] {
    const char* e = getenv("CMSISDSP_MI355X_SYNC");
    if (e && !strcmp(e, "sync")) return 0;
    if (e && !strcmp(e, "spin")) return 1;
    return MI355X_SYNC_DEFAULT;
  }();
  return m;
}

DoneWord* done_word() {
  const int dev = cur_dev();
  t_res.touch();
  DoneWord& w = t_res.done[dev];
  if (!w.h) {
    void* p = nullptr;
    if (hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return nullptr;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
      (void)hipHostFree(p);
      return nullptr;
    }
    w.h = (volatile uint32_t*)p;
    w.d = (uint32_t*)d;
    *w.h = 0;
  }
  return &w;
}
}  // namespace

bool done_slot(uint32_t** dflag, uint32_t* seq) {
  if (sync_mode() != 1) return false;
  DoneWord* w = done_word();
  if (!w) return false;
  if (++w->seq == 0) ++w->seq;               // 0 means "no self-signalled work" (HostIO::finish)
  *dflag = w->d;
  *seq = w->seq;
  return true;
}

// How long a synchronous call spins (with a pause per poll) before it blocks in
// hipStreamSynchronize: the small calls the spin exists for finish in ~10 us; a long call
// (a large mat_mult or FIR) blocks after this instead of burning a core.
constexpr auto kSpinBudget = std::chrono::microseconds(200);

hipError_t wait_done(hipStream_t st, uint32_t seq) {
  DoneWord* w = done_word();
  if (w) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0;; ++i) {
      if (__atomic_load_n(w->h, __ATOMIC_ACQUIRE) == seq) return hipSuccess;
      __builtin_ia32_pause();
      if ((i & 63) == 63 && std::chrono::steady_clock::now() - t0 > kSpinBudget) break;
    }
  }
  return hipStreamSynchronize(st);   // a slow or failed call: block (this also reports errors)
}

hipError_t wait_stream(hipStream_t st) {
  uint32_t* d = nullptr;
  uint32_t v = 0;
  if (done_slot(&d, &v)) {
    if (done_flag_launch(d, v, st) == hipSuccess) return wait_done(st, v);
    (void)hipGetLastError();
  }
  return hipStreamSynchronize(st);
}

hipError_t HostIO::finish(uint32_t seq) {
  finished_ = true;
  hipError_t e = seq ? wait_done(st_, seq) : wait_stream(st_);
  if (e != hipSuccess) return e;
  for (int i = 0; i < nouts_; ++i) memcpy(outs_[i].host, outs_[i].pin, outs_[i].bytes);
  nouts_ = 0;
  return hipSuccess;
}

hipStream_t sync_stream() {
  const int dev = cur_dev();
  auto it = t_res.streams.find(dev);
  if (it != t_res.streams.end()) return it->second;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  t_res.touch();
  t_res.streams[dev] = s;
  return s;
}

void release_thread_resources() { t_res.release(); }
int live_thread_owners() { return g_live_owners.load(std::memory_order_relaxed); }

}  // namespace mi355x

extern "C" {
int arm_mi355x_last_error(void) { return mi355x::g_err; }
const char* arm_mi355x_last_error_string(void) { return mi355x::g_err_msg.c_str(); }
size_t arm_mi355x_table_cache_bytes(void) { return mi355x::blob_cache_bytes(); }
void arm_mi355x_set_table_cache_limit(size_t bytes) { mi355x::set_blob_cache_limit(bytes); }
void arm_mi355x_clear_error(void) { mi355x::clear_error(); }
void arm_mi355x_release_thread_resources(void) { mi355x::release_thread_resources(); }
int arm_mi355x_thread_resource_owners(void) { return mi355x::live_thread_owners(); }
}
