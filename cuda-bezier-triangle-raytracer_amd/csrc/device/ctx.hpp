// ctx.hpp -- the context (bzr_ctx of include/bzr.h): device, streams and the device buffers it owns.
// Shared by the translation units of the device half (trace.hip, frame_pack.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "bzr.h"

struct bzr_ctx {
  int device;
  hipStream_t own;
  hipStream_t stream;
  void *scratch = nullptr;  // staging for host-pointer calls
  size_t scratch_bytes = 0;
  void *work = nullptr;     // candidate lists + counts
  size_t work_bytes = 0;
  // The culled path's counters and histogram start every segment at zero.  A segment on the small-scan
  // path leaves them zero for the next one (k_scan_small clears the histogram it reads, k_finish the
  // counters), so the memset is skipped while the workspace and histogram size are unchanged.
  const uint32_t *zero_ctr = nullptr;  // workspace counters known zero, with histogram [0, zero_hn]
  uint32_t zero_hn = 0;
  bool timing = false;      // per-kernel event timing (bzr_ctx_timing)
  struct Mark {
    int kernel;
    hipEvent_t start, stop;
  };
  std::vector<Mark> marks;       // recorded, not yet reported
  std::vector<hipEvent_t> spare; // event pool
  hipEvent_t handoff = nullptr;  // orders a new stream after the previous one (bzr_ctx_set_stream)
  double ms[BZR_KERNEL_COUNT] = {};
  uint32_t calls[BZR_KERNEL_COUNT] = {};
  uint32_t chunk_cap = 0;                // staged-path rays per chunk (0: not yet sized, chunk_for)
  bool counting = false;                 // work counters (bzr_ctx_counters)
  unsigned long long *counters = nullptr;  // device [BZR_COUNTER_COUNT]
  unsigned long long *wave_clock = nullptr;  // test hook (bzr_debug_wave_clock): per k_trace wave, device
  uint32_t wave_clock_cap = 0;
  bool wave_clock_real = false;  // bzr_debug_wave_clock_rate: also s_memrealtime (4 words per wave)
  void *pack = nullptr;     // bzr_pack_frame: per-block survivor counts and offsets (compact layout)
  size_t pack_bytes = 0;
  // cost-ordered k_trace dispatch (trace.hip run_fused): each wave of a fused call writes its cost class;
  // three small kernels turn them into a longest-first order of the waves, which the next fused call of the
  // same size dispatches in.  sched: device [cap] cost bins | [cap] order | histogram | offsets.
  uint32_t *sched = nullptr;
  uint32_t sched_cap = 0;    // waves the buffer holds
  uint32_t sched_waves = 0;  // waves of the call whose order is ready (0: none)
  uint32_t sched_calls = 0;  // calls since the order was first built for this size (rebuilt every BZR_TRACE_SCHED_REFRESH)
  uint64_t sched_key = 0;    // the order's call: lens set and mode (a different call of the same size rebuilds it)
};

// BZR_RAYS_AOS (frame_pack.hip): n rays between the reference's [n][6] records and the kernels' [6][n] rows,
// device to device on `stream` (to_soa: src AoS -> dst rows; else rows -> AoS).  src and dst must not overlap.
hipError_t bzr_rays_relayout(hipStream_t stream, const float *src, float *dst, uint32_t n, bool to_soa);
// bzr_intersect_records (frame_pack.hip): hit rows [13][n] on the device -> n bzr_hit_record at `records` and the
// patch words at `patch` (may be null), on `stream`.
hipError_t bzr_hits_to_records(hipStream_t stream, const float *rows, uint32_t n, void *records, uint32_t *patch);
