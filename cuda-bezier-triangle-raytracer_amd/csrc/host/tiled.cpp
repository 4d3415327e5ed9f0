// tiled.cpp -- bzr_trace_tiled: the refraction chain (reference/test.cpp:376-401) over several
// devices from one process.  Tiles of consecutive rays are dealt round-robin to the contexts; each
// context's tiles are packed into one SoA batch, traced by bzr_trace_chain on that context's own
// host thread (one host thread per bzr_ctx, as bzr.h requires), and scattered back in input order.
// No collective: rays are independent, so each device's results go straight to host memory.
#include <algorithm>
#include <cstring>
#include <exception>
#include <string>
#include <thread>
#include <vector>

#include "bzr.h"

extern "C" void bzr_internal_set_error(const char *msg);

namespace {

bzr_status fail(bzr_status s, std::string const &msg) {
  bzr_internal_set_error(msg.c_str());
  return s;
}

// Copy `count` rays of a `rows`-row SoA (row stride `ld_from`) starting at `from` to position `to`
// of another SoA (row stride `ld_to`).
void copy_rows(float const *src, std::size_t ld_from, std::size_t from, float *dst, std::size_t ld_to,
               std::size_t to, std::size_t count, int rows) {
  for (int r = 0; r < rows; ++r)
    std::memcpy(dst + r * ld_to + to, src + r * ld_from + from, count * sizeof(float));
}

struct Share {  // one context's tiles, packed
  std::vector<std::size_t> first;  // first ray of each tile
  std::vector<uint32_t> count;     // rays in each tile
  std::size_t n = 0;
  std::vector<float> in, out;
  std::vector<uint32_t> status, segments;
  bzr_status result = BZR_OK;
  std::string error;
};

}  // namespace

extern "C" bzr_status bzr_trace_tiled(bzr_ctx *const *ctxs, uint32_t nctx, const bzr_mesh *const *lenses,
                                      const float *ri, uint32_t nlens, const float *rays, uint32_t n,
                                      uint32_t tile_rays, float *out_rays, uint32_t *out_status,
                                      uint32_t *out_segments, uint32_t flags) {
  if (nctx == 0 || !ctxs) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_trace_tiled: no contexts");
  for (uint32_t d = 0; d < nctx; ++d)
    if (!ctxs[d] || std::find(ctxs, ctxs + d, ctxs[d]) != ctxs + d)
      return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_trace_tiled: null or repeated context (one host thread per context)");
  if (!lenses || !ri || nlens == 0) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_trace_tiled: null lens list");
  if (tile_rays == 0) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_trace_tiled: tile_rays must be > 0");
  if (flags & BZR_DEVICE_PTRS) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_trace_tiled: host pointers only");
  if (n == 0) return BZR_OK;
  if (!rays || !out_rays || !out_status) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_trace_tiled: null buffer");

  std::vector<Share> share(nctx);
  const std::size_t tiles = (static_cast<std::size_t>(n) + tile_rays - 1) / tile_rays;
  for (std::size_t k = 0; k < tiles; ++k) {
    Share &s = share[k % nctx];
    const std::size_t first = k * tile_rays;
    const uint32_t count = static_cast<uint32_t>(std::min<std::size_t>(tile_rays, n - first));
    s.first.push_back(first);
    s.count.push_back(count);
    s.n += count;
  }
  auto trace = [&](uint32_t d) {
    Share &s = share[d];
    if (s.n == 0) return;
    s.in.resize(6 * s.n);
    s.out.resize(6 * s.n);
    s.status.resize(s.n);
    if (out_segments) s.segments.resize(s.n);
    std::size_t at = 0;
    for (std::size_t t = 0; t < s.first.size(); ++t) {
      copy_rows(rays, n, s.first[t], s.in.data(), s.n, at, s.count[t], 6);
      at += s.count[t];
    }
    s.result = bzr_trace_chain(ctxs[d], lenses + static_cast<std::size_t>(d) * nlens, ri, nlens, s.in.data(),
                               static_cast<uint32_t>(s.n), s.out.data(), s.status.data(),
                               out_segments ? s.segments.data() : nullptr, flags);
    if (s.result != BZR_OK) {
      s.error = bzr_last_error();  // thread-local: carried back to the caller's thread below
      return;
    }
    at = 0;
    for (std::size_t t = 0; t < s.first.size(); ++t) {
      copy_rows(s.out.data(), s.n, at, out_rays, n, s.first[t], s.count[t], 6);
      std::memcpy(out_status + s.first[t], s.status.data() + at, s.count[t] * sizeof(uint32_t));
      if (out_segments) std::memcpy(out_segments + s.first[t], s.segments.data() + at, s.count[t] * sizeof(uint32_t));
      at += s.count[t];
    }
  };
  auto work = [&](uint32_t d) {
    try {
      trace(d);
    } catch (std::exception const &e) {  // allocation failure on this thread
      share[d].result = BZR_ERR_OUT_OF_MEMORY;
      share[d].error = e.what();
    }
  };
  std::vector<std::thread> threads;
  try {
    for (uint32_t d = 1; d < nctx; ++d) threads.emplace_back(work, d);
    work(0);
  } catch (std::exception const &e) {  // thread creation failure
    for (auto &t : threads) t.join();
    return fail(BZR_ERR_OUT_OF_MEMORY, std::string("bzr_trace_tiled: ") + e.what());
  }
  for (auto &t : threads) t.join();
  for (uint32_t d = 0; d < nctx; ++d)
    if (share[d].result != BZR_OK)
      return fail(share[d].result, "bzr_trace_tiled: context " + std::to_string(d) + ": " + share[d].error);
  return BZR_OK;
}
