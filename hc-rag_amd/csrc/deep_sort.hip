// deep_sort.hip — the segmented radix sorts behind the deep top-k path (k > 2048: every row's
// exact key per query, hcrag_index.hip deep_topk) and the sort-based shard merge (g x k > 8192,
// hcr_merge_topk_device).  rocPRIM's segmented radix sort (through hipCUB) is a stable LSD
// sort: rows enter each segment in ascending order, so a descending sort on the exact score
// key keeps equal scores in ascending row order -- the (score desc, row asc) tie rule of the
// whole library.  Its own translation unit: the template instantiations compile in parallel.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "hcrag.h"
#include "host_common.h"

// Sort `num_segments` segments (begin offsets offs[s], end offs[s + 1]) of (u64 key, u32 value)
// pairs, ascending (descending = 0) or descending (1).  temp: caller-owned scratch (grown here).
int hcr_seg_sort_u64_u32(DevBuf& temp, const uint64_t* kin, uint64_t* kout, const uint32_t* vin,
                         uint32_t* vout, int num_items, int num_segments, const int* offs,
                         int descending, hipStream_t st) {
  size_t bytes = 0;
  if (descending)
    HIPC(hipcub::DeviceSegmentedRadixSort::SortPairsDescending(nullptr, bytes, kin, kout, vin, vout, num_items,
                                                               num_segments, offs, offs + 1, 0, 64, st));
  else
    HIPC(hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, bytes, kin, kout, vin, vout, num_items,
                                                     num_segments, offs, offs + 1, 0, 64, st));
  CHECK(temp.ensure(bytes));
  bytes = temp.bytes;
  if (descending)
    HIPC(hipcub::DeviceSegmentedRadixSort::SortPairsDescending(temp.p, bytes, kin, kout, vin, vout, num_items,
                                                               num_segments, offs, offs + 1, 0, 64, st));
  else
    HIPC(hipcub::DeviceSegmentedRadixSort::SortPairs(temp.p, bytes, kin, kout, vin, vout, num_items,
                                                     num_segments, offs, offs + 1, 0, 64, st));
  return HCR_OK;
}
