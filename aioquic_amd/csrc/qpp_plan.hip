// qpp_plan.hip -- bucketing of a packet batch by (suite, key slot) on the
// device (quic_pp.h, qpp_plan_*).  A server's batch interleaves connections
// (src/aioquic/asyncio/server.py:60-152); the packet kernels want each
// workgroup on one key slot and each launch on one cipher suite, so the plan
// sorts packet indices by (suite, slot) with a stable LSD radix sort
// (rocPRIM) over just the bits the table's capacity needs, counts each
// suite's bucket, and gathers descriptors into that order for every launch.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <stdlib.h>

#include "qpp_internal.h"

namespace qpp {

constexpr int kPlanWG = 256;
constexpr uint32_t kNoKeyBucket = 3;  // empty or out-of-range slot: QPP_S_NO_KEY

// Sort key of packet i: bucket (suite, or 3 for no key) above the slot bits;
// one LDS histogram per workgroup, then four global adds.
__global__ __launch_bounds__(kPlanWG) void k_plan_keys(const KeySlot *__restrict__ slots, uint32_t cap,
                                                       const qpp_desc *__restrict__ desc, uint32_t n,
                                                       int slot_bits, uint32_t *__restrict__ keys,
                                                       uint32_t *__restrict__ idx,
                                                       uint32_t *__restrict__ count)
{
    __shared__ uint32_t hist[4];
    if (threadIdx.x < 4) hist[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * kPlanWG + threadIdx.x;
    if (i < n) {
        const uint32_t s = desc[i].slot;
        uint32_t b = kNoKeyBucket;
        if (s < cap) {
            const uint32_t suite = slots[s].suite;
            if (suite <= QPP_CHACHA20_POLY1305) b = suite;
        }
        keys[i] = b << slot_bits | (s < cap ? s : 0u);
        idx[i] = i;
        atomicAdd(&hist[b], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 4 && hist[threadIdx.x]) atomicAdd(&count[threadIdx.x], hist[threadIdx.x]);
}

// count[4] -> range[8] = [begin, end) of each bucket in sorted order
__global__ void k_plan_ranges(const uint32_t *__restrict__ count, uint32_t *__restrict__ range)
{
    if (threadIdx.x != 0) return;
    uint32_t b = 0;
    for (int s = 0; s < 4; ++s) {
        range[2 * s] = b;
        b += count[s];
        range[2 * s + 1] = b;
    }
}

constexpr uint32_t kItemPackets = 16;  // packets per wave in the packet kernels

// flags[p] = 1 where sorted position p starts a wave item: its offset from the
// start of its key's run (found by binary search in the sorted keys) is a
// multiple of 16.
__global__ __launch_bounds__(kPlanWG) void k_plan_heads(const uint32_t *__restrict__ skeys, uint32_t n,
                                                        uint32_t *__restrict__ flags)
{
    const uint32_t p = blockIdx.x * kPlanWG + threadIdx.x;
    if (p >= n) return;
    const uint32_t k = skeys[p];
    uint32_t lo = 0, hi = p;  // first position holding k lies in [lo, hi]
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (skeys[mid] < k) lo = mid + 1;
        else hi = mid;
    }
    flags[p] = ((p - lo) % kItemPackets) == 0 ? 1u : 0u;
}

// items[pos[p]] = p at every head; the last thread writes the sentinel and the
// item count
__global__ __launch_bounds__(kPlanWG) void k_plan_items(const uint32_t *__restrict__ flags,
                                                        const uint32_t *__restrict__ pos, uint32_t n,
                                                        uint32_t *__restrict__ items,
                                                        uint32_t *__restrict__ total)
{
    const uint32_t p = blockIdx.x * kPlanWG + threadIdx.x;
    if (p >= n) return;
    const uint32_t f = flags[p], i = pos[p];
    if (f) items[i] = p;
    if (p == n - 1) {
        items[i + f] = n;
        *total = i + f;
    }
}

// range[8] (positions) -> irange[8] (items): a bucket starts on an item head
__global__ void k_plan_iranges(const uint32_t *__restrict__ range, const uint32_t *__restrict__ pos,
                               const uint32_t *__restrict__ total, uint32_t n,
                               uint32_t *__restrict__ irange)
{
    if (threadIdx.x >= 8) return;
    const uint32_t r = range[threadIdx.x];
    irange[threadIdx.x] = r < n ? pos[r] : *total;
}

// ---- counting-sort path (tables of <= kPlanCountSlots slots) -------------
//
// keys -> per-key counts (bins) -> one-workgroup scan of the bins (each key's
// first position and first wave item; bucket ranges) -> wave items -> each
// packet's position: its rank within its workgroup's packets of that key plus
// the range the workgroup took from the key's cursor.
// Packets of one key keep no particular order among themselves (the results
// go back to the caller's order through rsv, so the order is not observable).

constexpr int kScanWG = 1024;
constexpr int kCntPer = 4;  // packets per thread of k_cnt_keys / k_cnt_scatter
constexpr uint32_t kMaxBins = 4u << 12;  // 4 buckets x 4096 slots (kPlanCountSlots)

__device__ __forceinline__ uint32_t plan_key(const KeySlot *slots, uint32_t cap, uint32_t s, int slot_bits)
{
    uint32_t b = kNoKeyBucket;
    if (s < cap) {
        const uint32_t suite = slots[s].suite;
        if (suite <= QPP_CHACHA20_POLY1305) b = suite;
    }
    return b << slot_bits | (s < cap ? s : 0u);
}

// Per-key counts: a workgroup of kCntPer x kScanWG packets counts its keys in
// an LDS histogram, then adds each non-zero bin to the global one (a batch on
// one connection would otherwise serialize its atomics on one address).  The
// histogram's clearing and flushing cost the same for any number of packets,
// so a workgroup takes several per thread.
__global__ __launch_bounds__(kScanWG) void k_cnt_keys(const KeySlot *__restrict__ slots, uint32_t cap,
                                                      const qpp_desc *__restrict__ desc, uint32_t n,
                                                      int slot_bits, uint32_t nb, uint32_t *__restrict__ keys,
                                                      uint32_t *__restrict__ bins)
{
    __shared__ uint32_t h[kMaxBins];
    for (uint32_t b = threadIdx.x; b < nb; b += kScanWG) h[b] = 0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kCntPer; ++u) {
        const uint32_t i = (blockIdx.x * kCntPer + u) * kScanWG + threadIdx.x;
        if (i < n) {
            const uint32_t k = plan_key(slots, cap, desc[i].slot, slot_bits);
            keys[i] = k;
            atomicAdd(&h[k], 1u);
        }
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += kScanWG)
        if (h[b]) atomicAdd(&bins[b], h[b]);
}

// One workgroup: bins[nb] counts -> posoff / itmoff (exclusive scans of the
// counts and of their wave items), bins[] = posoff (the scatter cursors),
// range / irange per bucket, count[24] = wave items in all, items[total] = n.
// Each thread scans a contiguous run of bins; the LDS copies are padded by one
// word per 32 (index b + b / 32) so that the threads' runs of 16 hit distinct
// banks, and every global read and write is coalesced through them.
__device__ __forceinline__ uint32_t scan_pad(uint32_t b) { return b + (b >> 5); }

__global__ __launch_bounds__(kScanWG) void k_cnt_scan(uint32_t *__restrict__ bins, uint32_t nb, int slot_bits,
                                                      uint32_t n, uint32_t *__restrict__ posoff,
                                                      uint32_t *__restrict__ itmoff,
                                                      uint32_t *__restrict__ count, uint32_t *__restrict__ items)
{
    __shared__ uint32_t c[kMaxBins + kMaxBins / 32], it[kMaxBins + kMaxBins / 32];
    __shared__ uint32_t sp[kScanWG], si[kScanWG];
    for (uint32_t b = threadIdx.x; b < nb; b += kScanWG) c[scan_pad(b)] = bins[b];
    __syncthreads();
    const uint32_t per = (nb + kScanWG - 1) / kScanWG, b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
    uint32_t tp = 0, ti = 0;
    for (uint32_t b = b0; b < b1; ++b) {
        const uint32_t v = c[scan_pad(b)];
        tp += v;
        ti += (v + kItemPackets - 1) / kItemPackets;
    }
    sp[threadIdx.x] = tp;
    si[threadIdx.x] = ti;
    __syncthreads();
    // inclusive Hillis-Steele scan of the per-thread sums
    for (int d = 1; d < kScanWG; d <<= 1) {
        const uint32_t ap = threadIdx.x >= (uint32_t)d ? sp[threadIdx.x - d] : 0u;
        const uint32_t ai = threadIdx.x >= (uint32_t)d ? si[threadIdx.x - d] : 0u;
        __syncthreads();
        sp[threadIdx.x] += ap;
        si[threadIdx.x] += ai;
        __syncthreads();
    }
    uint32_t pos = sp[threadIdx.x] - tp, itm = si[threadIdx.x] - ti;
    const uint32_t total = si[kScanWG - 1];
    const uint32_t smask = (1u << slot_bits) - 1;
    for (uint32_t b = b0; b < b1; ++b) {
        if ((b & smask) == 0) {
            // first bin of bucket b >> slot_bits: the bucket's start, the previous bucket's end
            const uint32_t s = b >> slot_bits;
            count[8 + 2 * s] = pos;
            count[16 + 2 * s] = itm;
            if (s > 0) {
                count[8 + 2 * s - 1] = pos;
                count[16 + 2 * s - 1] = itm;
            }
        }
        const uint32_t v = c[scan_pad(b)];
        c[scan_pad(b)] = pos;
        it[scan_pad(b)] = itm;
        pos += v;
        itm += (v + kItemPackets - 1) / kItemPackets;
    }
    if (threadIdx.x == 0) {
        count[8 + 7] = n;
        count[16 + 7] = total;
        count[24] = total;
        items[total] = n;
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += kScanWG) {
        const uint32_t v = c[scan_pad(b)];
        posoff[b] = v;
        bins[b] = v;
        itmoff[b] = it[scan_pad(b)];
    }
}

// items[j] = first sorted position of wave item j (j < total)
__global__ __launch_bounds__(kPlanWG) void k_cnt_items(const uint32_t *__restrict__ posoff,
                                                       const uint32_t *__restrict__ itmoff, uint32_t nb,
                                                       const uint32_t *__restrict__ count,
                                                       uint32_t *__restrict__ items)
{
    const uint32_t j = blockIdx.x * kPlanWG + threadIdx.x;
    if (j >= count[24]) return;
    // the last bin whose first item is <= j holds item j
    uint32_t lo = 0, hi = nb - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (itmoff[mid] <= j) lo = mid;
        else hi = mid - 1;
    }
    items[j] = posoff[lo] + kItemPackets * (j - itmoff[lo]);
}

// idx[position] = caller index.  Each workgroup ranks its packets per key in
// LDS, takes one range per non-zero key from the key's cursor (one global
// atomic per key and workgroup, all in flight together), and scatters.
__global__ __launch_bounds__(kScanWG) void k_cnt_scatter(const uint32_t *__restrict__ keys, uint32_t n,
                                                         uint32_t nb, uint32_t *__restrict__ cursor,
                                                         uint32_t *__restrict__ idx)
{
    constexpr int kPer = kMaxBins / kScanWG;  // bins per thread
    __shared__ uint32_t h[kMaxBins];
    for (uint32_t b = threadIdx.x; b < nb; b += kScanWG) h[b] = 0;
    __syncthreads();
    uint32_t k[kCntPer], r[kCntPer];
#pragma unroll
    for (int u = 0; u < kCntPer; ++u) {
        const uint32_t i = (blockIdx.x * kCntPer + u) * kScanWG + threadIdx.x;
        k[u] = i < n ? keys[i] : 0u;
        r[u] = i < n ? atomicAdd(&h[k[u]], 1u) : 0u;
    }
    __syncthreads();
    uint32_t base[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        const uint32_t b = threadIdx.x + u * kScanWG;
        const uint32_t c = b < nb ? h[b] : 0u;
        base[u] = c ? atomicAdd(&cursor[b], c) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        const uint32_t b = threadIdx.x + u * kScanWG;
        if (b < nb) h[b] = base[u];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kCntPer; ++u) {
        const uint32_t i = (blockIdx.x * kCntPer + u) * kScanWG + threadIdx.x;
        if (i < n) idx[h[k[u]] + r[u]] = i;
    }
}

// sorted[p] = desc[idx[p]], with the caller's index in rsv
__global__ __launch_bounds__(kPlanWG) void k_plan_gather(const qpp_desc *__restrict__ desc,
                                                         const uint32_t *__restrict__ idx, uint32_t n,
                                                         qpp_desc *__restrict__ sorted)
{
    const uint32_t p = blockIdx.x * kPlanWG + threadIdx.x;
    if (p >= n) return;
    const uint32_t i = idx[p];
    qpp_desc d = desc[i];
    d.rsv = i;
    sorted[p] = d;
}

// Results of the no-key bucket (KeyUnavailableError, quic/crypto.py:78-79):
// a grid-stride loop over [range[6], range[7]) with a small fixed grid.
__global__ __launch_bounds__(kPlanWG) void k_plan_nokey(const qpp_desc *__restrict__ sorted,
                                                        const uint32_t *__restrict__ range,
                                                        qpp_result *__restrict__ res)
{
    const uint32_t b = range[2 * kNoKeyBucket], e = range[2 * kNoKeyBucket + 1];
    for (uint32_t p = b + blockIdx.x * kPlanWG + threadIdx.x; p < e; p += gridDim.x * kPlanWG) {
        const qpp_desc d = sorted[p];
        res[d.rsv] = qpp_result{d.pn, QPP_S_NO_KEY, 0, 0};
    }
}

}  // namespace qpp

using namespace qpp;

static int bits_for(uint32_t cap)
{
    int b = 1;
    while (b < 24 && (1u << b) < cap) ++b;
    return b;
}

extern "C" int qpp_plan_create(uint32_t max_packets, qpp_plan **out)
{
    if (!out || max_packets == 0 || max_packets > (1u << 30)) return QPP_E_ARG;
    *out = NULL;
    qpp_plan *p = (qpp_plan *)calloc(1, sizeof(qpp_plan));
    if (!p) return QPP_E_NOMEM;
    p->cap = max_packets;
    const size_t n = max_packets;
    bool ok = hipMalloc(&p->d_keys[0], n * 4) == hipSuccess && hipMalloc(&p->d_keys[1], n * 4) == hipSuccess &&
              hipMalloc(&p->d_idx[0], n * 4) == hipSuccess && hipMalloc(&p->d_idx[1], n * 4) == hipSuccess &&
              hipMalloc(&p->d_sorted, n * sizeof(qpp_desc)) == hipSuccess &&
              hipMalloc(&p->d_flags, n * 4) == hipSuccess && hipMalloc(&p->d_pos, n * 4) == hipSuccess &&
              hipMalloc(&p->d_items, (n + 1) * 4) == hipSuccess &&
              hipMalloc(&p->d_count, 32 * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&p->d_bins, kMaxBins * 4) == hipSuccess && hipMalloc(&p->d_posoff, kMaxBins * 4) == hipSuccess &&
              hipMalloc(&p->d_itmoff, kMaxBins * 4) == hipSuccess;
    if (ok) {
        size_t tmp = 0, tmp2 = 0;
        ok = rocprim::radix_sort_pairs(nullptr, tmp, p->d_keys[0], p->d_keys[1], p->d_idx[0], p->d_idx[1],
                                       max_packets, 0, 26) == hipSuccess &&
             rocprim::exclusive_scan(nullptr, tmp2, p->d_flags, p->d_pos, 0u, max_packets,
                                     rocprim::plus<uint32_t>()) == hipSuccess;
        if (tmp2 > tmp) tmp = tmp2;
        ok = ok && hipMalloc(&p->d_tmp, tmp ? tmp : 16) == hipSuccess;
        p->tmp_bytes = tmp;
    }
    if (!ok) {
        (void)hipGetLastError();
        qpp_plan_destroy(p);
        return QPP_E_NOMEM;
    }
    p->d_range = p->d_count + 8;
    p->d_irange = p->d_count + 16;
    *out = p;
    return QPP_OK;
}

extern "C" void qpp_plan_destroy(qpp_plan *p)
{
    if (!p) return;
    for (int i = 0; i < 2; ++i) {
        if (p->d_keys[i]) (void)hipFree(p->d_keys[i]);
        if (p->d_idx[i]) (void)hipFree(p->d_idx[i]);
    }
    if (p->d_sorted) (void)hipFree(p->d_sorted);
    if (p->d_count) (void)hipFree(p->d_count);
    if (p->d_flags) (void)hipFree(p->d_flags);
    if (p->d_pos) (void)hipFree(p->d_pos);
    if (p->d_items) (void)hipFree(p->d_items);
    if (p->d_tmp) (void)hipFree(p->d_tmp);
    if (p->d_bins) (void)hipFree(p->d_bins);
    if (p->d_posoff) (void)hipFree(p->d_posoff);
    if (p->d_itmoff) (void)hipFree(p->d_itmoff);
    free(p);
}

int qpp_internal_plan_build(qpp_plan *p, const KeySlot *d_slots, uint32_t cap, const qpp_desc *d_desc,
                            uint32_t n, hipStream_t s)
{
    if (n > p->cap) return QPP_E_ARG;
    if (hipMemsetAsync(p->d_count, 0, 32 * sizeof(uint32_t), s) != hipSuccess) return QPP_E_HIP;
    const int sb = bits_for(cap);
    const dim3 grid((n + kPlanWG - 1) / kPlanWG);
    if (n && cap <= kPlanCountSlots && getenv("QPP_PLAN_RADIX") == nullptr) {
        const uint32_t nb = 4u << sb;
        if (hipMemsetAsync(p->d_bins, 0, nb * 4, s) != hipSuccess) return QPP_E_HIP;
        const dim3 cgrid((n + kCntPer * kScanWG - 1) / (kCntPer * kScanWG));
        hipLaunchKernelGGL(k_cnt_keys, cgrid, dim3(kScanWG), 0, s, d_slots, cap, d_desc, n, sb, nb, p->d_keys[0],
                           p->d_bins);
        hipLaunchKernelGGL(k_cnt_scan, dim3(1), dim3(kScanWG), 0, s, p->d_bins, nb, sb, n, p->d_posoff,
                           p->d_itmoff, p->d_count, p->d_items);
        const uint32_t mi = qpp_internal_plan_max_items(n, cap);
        hipLaunchKernelGGL(k_cnt_items, dim3((mi + kPlanWG - 1) / kPlanWG), dim3(kPlanWG), 0, s, p->d_posoff,
                           p->d_itmoff, nb, p->d_count, p->d_items);
        hipLaunchKernelGGL(k_cnt_scatter, cgrid, dim3(kScanWG), 0, s, p->d_keys[0], n, nb, p->d_bins, p->d_idx[1]);
        if (hipGetLastError() != hipSuccess) return QPP_E_HIP;
        p->n_built = n;
        return QPP_OK;
    }
    if (n) {
        hipLaunchKernelGGL(k_plan_keys, grid, dim3(kPlanWG), 0, s, d_slots, cap, d_desc, n, sb, p->d_keys[0],
                           p->d_idx[0], p->d_count);
        size_t tmp = p->tmp_bytes;
        if (rocprim::radix_sort_pairs(p->d_tmp, tmp, p->d_keys[0], p->d_keys[1], p->d_idx[0], p->d_idx[1], n,
                                      0, sb + 2, s) != hipSuccess)
            return QPP_E_HIP;
        hipLaunchKernelGGL(k_plan_heads, grid, dim3(kPlanWG), 0, s, p->d_keys[1], n, p->d_flags);
        tmp = p->tmp_bytes;
        if (rocprim::exclusive_scan(p->d_tmp, tmp, p->d_flags, p->d_pos, 0u, n, rocprim::plus<uint32_t>(),
                                    s) != hipSuccess)
            return QPP_E_HIP;
        hipLaunchKernelGGL(k_plan_items, grid, dim3(kPlanWG), 0, s, p->d_flags, p->d_pos, n, p->d_items,
                           p->d_count + 24);
    }
    hipLaunchKernelGGL(k_plan_ranges, dim3(1), dim3(64), 0, s, p->d_count, p->d_range);
    if (n) hipLaunchKernelGGL(k_plan_iranges, dim3(1), dim3(64), 0, s, p->d_range, p->d_pos, p->d_count + 24, n,
                              p->d_irange);
    if (hipGetLastError() != hipSuccess) return QPP_E_HIP;
    p->n_built = n;
    return QPP_OK;
}

int qpp_internal_plan_gather(const qpp_plan *p, const qpp_desc *d_desc, uint32_t n, hipStream_t s)
{
    if (n != p->n_built) return QPP_E_ARG;
    if (n == 0) return QPP_OK;
    hipLaunchKernelGGL(k_plan_gather, dim3((n + kPlanWG - 1) / kPlanWG), dim3(kPlanWG), 0, s, d_desc,
                       p->d_idx[1], n, p->d_sorted);
    return hipGetLastError() == hipSuccess ? QPP_OK : QPP_E_HIP;
}

uint32_t qpp_internal_plan_max_items(uint32_t n, uint32_t cap)
{
    // every key run adds at most one partial item; runs <= distinct slots
    // + the no-key bucket
    const uint64_t m = (uint64_t)(n + kItemPackets - 1) / kItemPackets + (n < cap ? n : cap) + 1;
    return (uint32_t)(m < n ? m : n);
}

int qpp_internal_plan_nokey(const qpp_plan *p, qpp_result *d_res, hipStream_t s)
{
    hipLaunchKernelGGL(k_plan_nokey, dim3(16), dim3(kPlanWG), 0, s, p->d_sorted, p->d_range, d_res);
    return hipGetLastError() == hipSuccess ? QPP_OK : QPP_E_HIP;
}
