// qpp_internal.h -- library-internal interfaces between the translation units
// of libquicpp.so (not part of the C ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "qpp_device.h"

// A batch's bucketing (quic_pp.h, qpp_plan_*): device buffers for n <= cap.
struct qpp_plan {
    uint32_t cap;
    uint32_t n_built;            // packets of the last qpp_plan_build
    uint32_t *d_keys[2];         // sort keys (bucket << slot_bits | slot), in / out
    uint32_t *d_idx[2];          // packet indices, in / sorted
    qpp_desc *d_sorted;          // descriptors gathered into bucket order (rsv = caller index)
    uint32_t *d_count;           // [0, 4): packets per bucket; [8, 16): d_range; [16, 24): d_irange;
                                 // [24]: wave items in all
    uint32_t *d_range;           // [begin, end) per bucket: AES-128, AES-256, ChaCha20, no key
    // Wave items: runs of <= 16 sorted positions on one key slot, so that no
    // wave of a packet kernel (16 packets, 4 lanes each) straddles two slots.
    // item i = positions [d_items[i], d_items[i + 1]); d_items[total] = n.
    uint32_t *d_flags;           // 1 where a position starts an item
    uint32_t *d_pos;             // exclusive scan of d_flags: item index of a head
    uint32_t *d_items;           // item start positions (+ the sentinel n)
    uint32_t *d_irange;          // [begin, end) of each bucket's items
    void *d_tmp;                 // rocPRIM temporary storage
    size_t tmp_bytes;
    // Counting-sort path (tables of <= kPlanCountSlots slots): one bin per
    // sort key, 4 << slot_bits bins.
    uint32_t *d_bins;            // per-key counts, then the scatter cursors
    uint32_t *d_posoff;          // first sorted position of each key's run
    uint32_t *d_itmoff;          // first wave item of each key's run
};

// Tables up to this many slots bucket by a counting sort over (suite, slot)
// keys; larger ones by the rocPRIM radix sort.
constexpr uint32_t kPlanCountSlots = 4096;

int qpp_internal_plan_build(qpp_plan *p, const qpp::KeySlot *d_slots, uint32_t cap,
                            const qpp_desc *d_desc, uint32_t n, hipStream_t s);
int qpp_internal_plan_gather(const qpp_plan *p, const qpp_desc *d_desc, uint32_t n, hipStream_t s);
// wave items of a batch of n packets on a table of `cap` slots, at most
uint32_t qpp_internal_plan_max_items(uint32_t n, uint32_t cap);
int qpp_internal_plan_nokey(const qpp_plan *p, qpp_result *d_res, hipStream_t s);
