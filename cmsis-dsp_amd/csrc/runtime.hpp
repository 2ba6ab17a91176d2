// Host runtime of the MI355X CMSIS-DSP backend: devices, streams, the device-side table
// cache, staging buffers for the host-pointer (drop-in) API and the error channel.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace mi355x {

// Thread-local error channel: processing functions of the reference return void, so a
// device failure is recorded here (arm_mi355x_last_error) instead of aborting.
void set_error(hipError_t e, const char* where);
void clear_error();

// True when p is device-accessible HIP memory (hipMalloc / managed).  Host memory,
// including hipHostMalloc'd pinned memory, is staged through a device scratch buffer.
bool is_device_ptr(const void* p);

// True when p lies inside this library's own image (its CommonTables / const instances):
// those words never change, so their device copies are cached by address.
bool is_library_addr(const void* p);

// Device view of a table (twiddles, RFFT twiddles, coefficients):
//   * a device pointer is used in place (no copy; the caller keeps it alive);
//   * the library's own tables are uploaded once per (device, address);
//   * any other host table is cached by CONTENT (device_blob), so a caller that frees a
//     table and reuses the address for new values never gets a stale copy.
// Returns nullptr on failure.
const void* device_table(const void* host, size_t bytes);

// Device copy of a host byte blob, cached by CONTENT (hash + full compare): uploaded once
// per distinct contents and device, immune to a caller reusing a buffer for new values.
// Used for user-supplied tables and coefficients (FIR taps, MFCC filterbanks, ...).  The
// cache is an LRU bounded in bytes per device (blob_cache_bytes / set_blob_cache_limit): a
// caller that changes coefficients on every call cycles through it instead of growing it.
// The returned pointer stays valid while the calling thread's innermost BlobScope lives and
// until the work enqueued before that scope ended has completed.  Returns nullptr on failure.
const void* device_blob(const void* host, size_t bytes);
size_t blob_cache_bytes();

// Device table of the fixed-point RFFT split's per-bin twiddle records, bin k < L:
// {A[2 mod k], A[2 mod k + 1], B[2 mod k], B[2 mod k + 1]} (arm_rfft_q31.c:293-326 index), `elem`
// bytes per word (4: int4 records, 2: 8-B records), so that a split reads one record per bin
// instead of four words at a stride of 2 mod (rfft_fixed_split.hpp SplitRecTab).  The library's own tables: built once per (device,
// A, B, mod, L); any other (host or device) table: rebuilt per call and cached by content.
// *symmetric (optional): record L - k equals record k with A1 and B1 negated for every k (true of the
// reference's realCoefA/B tables), which the fused N = 8192 q31 inverse relies on.
// A device-resident table is read back on `st` (the call's stream, then synchronized), so a table
// the caller wrote on that stream just before the call is read after that write.
const void* device_split_records(const void* A, const void* B, uint32_t mod, uint32_t L, int elem, hipStream_t st,
                                 bool* symmetric = nullptr);
void set_blob_cache_limit(size_t bytes);   // per device

// Pins every blob device_blob / device_table / device_perm hand out on this thread while the
// scope lives (eviction skips held blobs), then records one event on `st` -- after the work the
// call enqueued -- that the blobs' eventual release waits on (stream-ordered hipFreeAsync, no
// device synchronize).  Declare one in every entry point that fetches tables, before the first
// fetch, with the stream its launches go to; scopes nest (the innermost holds).
class BlobScope {
 public:
  explicit BlobScope(hipStream_t st);
  ~BlobScope();
  // the work this scope enqueued has completed (a synchronous call after its wait): the held
  // blobs are released without recording an event
  void synced() { synced_ = true; }
  BlobScope(const BlobScope&) = delete;
  BlobScope& operator=(const BlobScope&) = delete;

 private:
  hipStream_t st_;
  size_t base_;
  int dev_;
  bool synced_ = false;
};

// Device permutation implementing a bit-reversal swap table of a non-canonical instance.
// *canonical is set when the table induces the reference's own permutation (then the
// kernels compute it on the fly and nullptr is returned).  kind: 0 = f32 tables
// (mixed-radix digit reversal), 1 = fixed-point tables (binary bit reversal).
const uint16_t* device_perm(int n, const uint16_t* table, uint16_t len, int kind, bool* canonical, bool* ok);

// Per-thread device scratch for the synchronous host-pointer path (grown on demand).
void* scratch(size_t bytes, int slot);

// Per-thread pinned (hipHostMalloc) bounce buffer, grown on demand.
void* pinned(size_t bytes, int slot);

// Host <-> device staging of one synchronous drop-in call: host words are copied into a
// pinned bounce buffer and DMA'd from there (in), device results are DMA'd into a pinned
// buffer and copied to the caller's memory after the stream has drained (finish).  One
// pinned slot per transfer; a call ends with finish(), or the destructor drains the stream
// (error returns), so the slots are free again for the next call.
//
// Small calls (kZeroCopyMax bytes per buffer) skip the DMA engines: zin / zout / zinout return
// a COHERENT pinned buffer (hipHostMallocCoherent: the GPU reads and writes it directly over the
// host link, uncached, so no stale line survives between calls) holding the caller's words, the
// kernel runs on it in place, and finish() copies the results back -- one launch and one
// synchronize per call instead of two copies around the launch (tools/latency/).
constexpr size_t kZeroCopyMax = size_t(1) << 20;
class HostIO {
 public:
  explicit HostIO(hipStream_t st) : st_(st) {}
  ~HostIO();
  HostIO(const HostIO&) = delete;
  HostIO& operator=(const HostIO&) = delete;
  hipError_t in(void* dev, const void* host, size_t bytes);
  hipError_t out(void* host, const void* dev, size_t bytes);
  void* zin(const void* host, size_t bytes);                 // nullptr: allocation failed
  void* zout(void* host, size_t bytes);
  void* zinout(void* host, size_t bytes);
  hipError_t finish(uint32_t seq = 0);   // seq != 0: the work signals completion itself

 private:
  struct Pending { void* host; const void* pin; size_t bytes; };
  hipStream_t st_;
  int slot_ = 0, zslot_ = 0;
  Pending outs_[6];
  int nouts_ = 0;
  bool finished_ = false;
};

// Wait for everything enqueued on st (the synchronous drop-in calls' completion): a spin on a
// host word written by the stream, or hipStreamSynchronize (runtime.cpp, CMSISDSP_MI355X_SYNC).
hipError_t wait_stream(hipStream_t st);

// Spin mode: the calling thread's completion word on the current device and the next sequence
// number, for a launch that signals its own completion (common.hpp signal_done) -- one launch per
// call instead of the work plus done_flag_launch.  false in sync mode or when unavailable.
bool done_slot(uint32_t** dflag, uint32_t* seq);
// Wait until the completion word holds seq (bounded spin), then as wait_stream's fallback.
hipError_t wait_done(hipStream_t st, uint32_t seq);

// The internal stream used by the synchronous drop-in API on the current device.
hipStream_t sync_stream();

// Drain and free the calling thread's streams, scratch, staging and completion words (done
// automatically when a thread other than the main thread exits).  The next call re-creates them.
void release_thread_resources();
// Number of threads currently holding per-thread runtime resources.
int live_thread_owners();

}  // namespace mi355x
