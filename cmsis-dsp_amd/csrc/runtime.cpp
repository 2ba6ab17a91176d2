// Host runtime: device table cache, staging scratch, error channel.
#include "runtime.hpp"

#include <dlfcn.h>
#include <link.h>
#include <string.h>

#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/arm_math_mi355x.h"

namespace mi355x {

namespace {
thread_local int g_err = 0;
thread_local std::string g_err_msg;

std::mutex g_table_mu;
std::map<std::tuple<int, const void*, size_t>, void*> g_tables;
std::map<std::tuple<int, const void*, uint16_t, int, int>, std::pair<void*, bool>> g_perms;

// Content-keyed blob cache, bounded: an LRU by bytes per process (default 256 MiB, set with
// arm_mi355x_set_table_cache_limit).  Evicting synchronizes the device before hipFree, since
// an asynchronous batched call may still be reading the blob on any stream.
struct Blob { std::vector<uint8_t> host; void* dev = nullptr; int d = 0; uint64_t tick = 0; };
std::map<std::tuple<int, uint64_t, size_t>, std::vector<Blob>> g_blobs;
size_t g_blob_bytes = 0;
size_t g_blob_limit = size_t(256) << 20;
uint64_t g_blob_tick = 0;

// evict least-recently-used blobs until `incoming` more bytes fit (caller holds g_table_mu)
void blob_evict(size_t incoming) {
  while (g_blob_bytes + incoming > g_blob_limit && g_blob_bytes > 0) {
    auto victim_bucket = g_blobs.end();
    size_t victim = 0;
    uint64_t oldest = UINT64_MAX;
    for (auto it = g_blobs.begin(); it != g_blobs.end(); ++it)
      for (size_t i = 0; i < it->second.size(); ++i)
        if (it->second[i].tick < oldest) { oldest = it->second[i].tick; victim_bucket = it; victim = i; }
    if (victim_bucket == g_blobs.end()) break;
    Blob& b = victim_bucket->second[victim];
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != b.d) (void)hipSetDevice(b.d);
    (void)hipDeviceSynchronize();           // no kernel may still read it
    (void)hipFree(b.dev);
    if (prev != b.d) (void)hipSetDevice(prev);
    g_blob_bytes -= b.host.size();
    victim_bucket->second.erase(victim_bucket->second.begin() + (long)victim);
    if (victim_bucket->second.empty()) g_blobs.erase(victim_bucket);
  }
}

uint64_t fnv1a(const uint8_t* p, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ull; }
  return h;
}

struct Scratch { void* p = nullptr; size_t n = 0; };
thread_local std::map<std::pair<int, int>, Scratch> g_scratch;
struct Pinned { void* p = nullptr; size_t n = 0; };   // kept until process exit, like Scratch
thread_local std::map<int, Pinned> g_pinned;
thread_local std::map<int, Pinned> g_zpinned;      // coherent, device-accessed in place
thread_local std::map<int, hipStream_t> g_streams;

int cur_dev() { int d = 0; (void)hipGetDevice(&d); return d; }

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
  std::lock_guard<std::mutex> lk(g_table_mu);
  {
    auto it = g_blobs.find(key);
    if (it != g_blobs.end())
      for (Blob& b : it->second)
        if (memcmp(b.host.data(), h, bytes) == 0) { b.tick = ++g_blob_tick; return b.dev; }
  }
  blob_evict(bytes);
  Blob b;
  b.host.assign(h, h + bytes);
  b.d = dev;
  b.tick = ++g_blob_tick;
  hipError_t e = hipMalloc(&b.dev, bytes);
  if (e != hipSuccess) { set_error(e, "device_blob: hipMalloc"); return nullptr; }
  e = hipMemcpy(b.dev, h, bytes, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    set_error(e, "device_blob: hipMemcpy");
    (void)hipFree(b.dev);
    return nullptr;
  }
  std::vector<Blob>& bucket = g_blobs[key];
  bucket.push_back(std::move(b));
  g_blob_bytes += bytes;
  return bucket.back().dev;
}

size_t blob_cache_bytes() {
  std::lock_guard<std::mutex> lk(g_table_mu);
  return g_blob_bytes;
}
void set_blob_cache_limit(size_t bytes) {
  std::lock_guard<std::mutex> lk(g_table_mu);
  g_blob_limit = bytes;
  blob_evict(0);
}

const uint16_t* device_perm(int n, const uint16_t* table, uint16_t len, int kind, bool* canonical, bool* ok) {
  *ok = true;
  *canonical = true;
  if (!table) { return nullptr; }
  const int dev = cur_dev();
  // the library's own tables are immutable: cache their verdict by address; any other
  // table is re-derived from its current words on every call (O(len)) and a non-canonical
  // permutation is uploaded through the content-keyed blob cache
  const bool lib = is_library_addr(table);
  auto key = std::make_tuple(dev, (const void*)table, len, kind, n);
  if (lib) {
    std::lock_guard<std::mutex> lk(g_table_mu);
    auto it = g_perms.find(key);
    if (it != g_perms.end()) {
      *canonical = it->second.second;
      return (const uint16_t*)it->second.first;
    }
  }
  // apply the reference's sequential swaps (arm_bitreversal2.c:84-108) to an identity
  // array of complex indices: a[pos] = pre-reversal index that ends up at pos.
  const uint16_t* host = table;
  std::vector<uint16_t> tmp;
  if (is_device_ptr(table)) {
    tmp.resize(len);
    if (hipMemcpy(tmp.data(), table, len * sizeof(uint16_t), hipMemcpyDeviceToHost) != hipSuccess) { *ok = false; return nullptr; }
    host = tmp.data();
  }
  std::vector<uint16_t> a(n);
  for (int i = 0; i < n; ++i) a[i] = (uint16_t)i;
  for (int i = 0; i + 1 < len; i += 2) {
    const int x = host[i] >> 3, y = host[i + 1] >> 3;
    if (x >= n || y >= n) { *ok = false; return nullptr; }
    std::swap(a[x], a[y]);
  }
  bool canon = true;
  for (int k = 0; k < n && canon; ++k) canon = a[k] == (kind == 0 ? f32_src(n, k) : fixed_src(n, k));
  const void* d = nullptr;
  if (!canon) {
    d = device_blob(a.data(), n * sizeof(uint16_t));
    if (!d) { *ok = false; return nullptr; }
  }
  if (lib) {
    std::lock_guard<std::mutex> lk(g_table_mu);
    g_perms[key] = {(void*)d, canon};
  }
  *canonical = canon;
  return (const uint16_t*)d;
}

void* scratch(size_t bytes, int slot) {
  const int dev = cur_dev();
  Scratch& s = g_scratch[{dev, slot}];
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
  Pinned& s = g_pinned[slot];
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
  Pinned& s = g_zpinned[slot];
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

hipError_t HostIO::finish() {
  finished_ = true;
  hipError_t e = hipStreamSynchronize(st_);
  if (e != hipSuccess) return e;
  for (int i = 0; i < nouts_; ++i) memcpy(outs_[i].host, outs_[i].pin, outs_[i].bytes);
  nouts_ = 0;
  return hipSuccess;
}

hipStream_t sync_stream() {
  const int dev = cur_dev();
  auto it = g_streams.find(dev);
  if (it != g_streams.end()) return it->second;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  g_streams[dev] = s;
  return s;
}

}  // namespace mi355x

extern "C" {
int arm_mi355x_last_error(void) { return mi355x::g_err; }
const char* arm_mi355x_last_error_string(void) { return mi355x::g_err_msg.c_str(); }
size_t arm_mi355x_table_cache_bytes(void) { return mi355x::blob_cache_bytes(); }
void arm_mi355x_set_table_cache_limit(size_t bytes) { mi355x::set_blob_cache_limit(bytes); }
void arm_mi355x_clear_error(void) { mi355x::clear_error(); }
}
