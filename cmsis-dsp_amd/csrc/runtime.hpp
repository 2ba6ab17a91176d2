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

// Device copy of an immutable host table (twiddles, RFFT twiddles), uploaded once per
// (device, host pointer, size).  Returns nullptr on failure.
const void* device_table(const void* host, size_t bytes);

// Device copy of a host byte blob, cached by CONTENT (hash + full compare): uploaded once
// per distinct contents and device, immune to a caller reusing a buffer for new values.
// Used for user-supplied coefficient tables (MFCC).  Returns nullptr on failure.
const void* device_blob(const void* host, size_t bytes);

// Device permutation implementing a bit-reversal swap table of a non-canonical instance.
// *canonical is set when the table induces the reference's own permutation (then the
// kernels compute it on the fly and nullptr is returned).  kind: 0 = f32 tables
// (mixed-radix digit reversal), 1 = fixed-point tables (binary bit reversal).
const uint16_t* device_perm(int n, const uint16_t* table, uint16_t len, int kind, bool* canonical, bool* ok);

// Per-thread device scratch for the synchronous host-pointer path (grown on demand).
void* scratch(size_t bytes, int slot);

// The internal stream used by the synchronous drop-in API on the current device.
hipStream_t sync_stream();

}  // namespace mi355x
