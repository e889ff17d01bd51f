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
    uint32_t *d_count;           // [0, 4): packets per bucket; [8, 16): d_range
    uint32_t *d_range;           // [begin, end) per bucket: AES-128, AES-256, ChaCha20, no key
    void *d_tmp;                 // rocPRIM temporary storage
    size_t tmp_bytes;
};

int qpp_internal_plan_build(qpp_plan *p, const qpp::KeySlot *d_slots, uint32_t cap,
                            const qpp_desc *d_desc, uint32_t n, hipStream_t s);
int qpp_internal_plan_gather(const qpp_plan *p, const qpp_desc *d_desc, uint32_t n, hipStream_t s);
int qpp_internal_plan_nokey(const qpp_plan *p, qpp_result *d_res, hipStream_t s);
