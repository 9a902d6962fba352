// Transaction pipeline glue for gfx950: from device-computed WireTransaction ids to the
// per-signature verify items (cg_verify_transactions*, include/cordagpu.h).
//
//   k_txsig_items   one lane per signature: a cg_item whose clear data is its slot in the
//                   spliced-message workspace (flag CG_ITEM_MSG_WS), or an out-of-range key
//                   index (-> CG_NOT_RUN) when its transaction has no id or its template /
//                   transaction index is invalid. tx_status == nullptr: the ids are the
//                   caller's (cg_verify_tx_signatures*), every one valid
//   k_splice        one lane per dword of every message slot: prefix || id || suffix, i.e.
//                   SignableData(id, metadata).serialize() (Crypto.kt:499-502) for the
//                   signature's metadata template; coalesced 4-byte stores
#include <hip/hip_runtime.h>

#include "engine.h"
#include "keyws.h"

namespace cg {

__device__ __forceinline__ bool tmpl_ok(const cg_signable_tmpl& t, uint64_t arena_len) {
  return in_arena(t.prefix_off, t.prefix_len, arena_len) && in_arena(t.suffix_off, t.suffix_len, arena_len);
}

__global__ void __launch_bounds__(256) k_txsig_items(const cg_txsig* __restrict__ sigs, uint64_t n_sigs,
                                                     const cg_signable_tmpl* __restrict__ tmpls, uint32_t n_tmpls,
                                                     const uint8_t* __restrict__ tx_status, uint64_t n_tx,
                                                     uint64_t arena_len, uint64_t slot,
                                                     cg_item* __restrict__ items) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_sigs) return;
  const cg_txsig s = sigs[j];
  cg_item it;
  it.sig_off = s.sig_off;
  it.sig_len = s.sig_len;
  it.reserved1 = 0;
  bool ok = s.tx_idx < n_tx && s.tmpl < n_tmpls;
  if (ok && tx_status) ok = tx_status[s.tx_idx] == 0;
  cg_signable_tmpl t = {0, 0, 0, 0};
  if (ok) {
    t = tmpls[s.tmpl];
    ok = tmpl_ok(t, arena_len);
  }
  if (ok) {
    it.msg_off = j * slot;
    it.msg_len = t.prefix_len + 32u + t.suffix_len;
    it.key_idx = s.key_idx;
    it.reserved0 = CG_ITEM_MSG_WS;
  } else {
    it.msg_off = 0;
    it.msg_len = 0;
    it.key_idx = 0xffffffffu;  // k_misc_status: CG_NOT_RUN
    it.reserved0 = 0;
  }
  items[j] = it;
}

__global__ void __launch_bounds__(256) k_splice(const cg_txsig* __restrict__ sigs, uint64_t n_sigs,
                                                const cg_signable_tmpl* __restrict__ tmpls, uint32_t n_tmpls,
                                                const uint8_t* __restrict__ tx_status, uint64_t n_tx,
                                                const uint8_t* __restrict__ ids, const uint8_t* __restrict__ arena,
                                                uint64_t arena_len, uint64_t slot, uint8_t* __restrict__ msgs) {
  const uint64_t wpr = slot >> 2;
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t j = g / wpr, w = g % wpr;
  if (j >= n_sigs) return;
  const cg_txsig s = sigs[j];
  uint32_t v = 0;
  if (s.tx_idx < n_tx && s.tmpl < n_tmpls && (!tx_status || tx_status[s.tx_idx] == 0)) {
    const cg_signable_tmpl t = tmpls[s.tmpl];
    if (tmpl_ok(t, arena_len)) {
      const uint64_t n = (uint64_t)t.prefix_len + 32u + t.suffix_len;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint64_t p = 4 * w + b;
        uint32_t byte = 0;
        if (p < t.prefix_len) byte = arena[t.prefix_off + p];
        else if (p < t.prefix_len + 32u) byte = ids[32 * (uint64_t)s.tx_idx + (p - t.prefix_len)];
        else if (p < n) byte = arena[t.suffix_off + (p - t.prefix_len - 32u)];
        v |= byte << (8 * b);
      }
    }
  }
  ((uint32_t*)msgs)[g] = v;
}

hipError_t launch_tx_sig_items(const cg_txsig* d_sigs, uint64_t n_sigs, const cg_signable_tmpl* d_tmpls,
                               uint32_t n_tmpls, const uint8_t* d_tx_status, uint64_t n_tx, const uint8_t* d_ids,
                               const uint8_t* d_arena, uint64_t arena_len, uint64_t slot, cg_item* d_items,
                               uint8_t* d_msgs, hipStream_t stream) {
  if (n_sigs == 0) return hipSuccess;
  const uint32_t B = 256;
  hipLaunchKernelGGL(k_txsig_items, dim3((unsigned)((n_sigs + B - 1) / B)), dim3(B), 0, stream, d_sigs, n_sigs,
                     d_tmpls, n_tmpls, d_tx_status, n_tx, arena_len, slot, d_items);
  const uint64_t words = n_sigs * (slot >> 2);
  hipLaunchKernelGGL(k_splice, dim3((unsigned)((words + B - 1) / B)), dim3(B), 0, stream, d_sigs, n_sigs, d_tmpls,
                     n_tmpls, d_tx_status, n_tx, d_ids, d_arena, arena_len, slot, d_msgs);
  return hipGetLastError();
}

}  // namespace cg
