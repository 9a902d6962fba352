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
#include "sha2.h"

namespace cg {

__device__ __forceinline__ bool tmpl_ok(const cg_signable_tmpl& t, uint64_t arena_len) {
  return in_arena(t.prefix_off, t.prefix_len, arena_len) && in_arena(t.suffix_off, t.suffix_len, arena_len);
}

__global__ void __launch_bounds__(256) k_txsig_items(const cg_txsig* __restrict__ sigs, uint64_t n_sigs,
                                                     const cg_signable_tmpl* __restrict__ tmpls, uint32_t n_tmpls,
                                                     const uint8_t* __restrict__ tx_status, uint64_t n_tx,
                                                     uint64_t arena_len, uint64_t head, uint64_t slot,
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
    it.msg_off = head + j * slot;
    it.msg_len = t.prefix_len + 32u + t.suffix_len;
    it.key_idx = s.key_idx;
    it.reserved0 = CG_ITEM_MSG_WS | CG_ITEM_TMPL;
    it.reserved1 = s.tmpl;
  } else {
    it.msg_off = 0;
    it.msg_len = 0;
    it.key_idx = 0xffffffffu;  // k_misc_status: CG_NOT_RUN
    it.reserved0 = 0;
  }
  items[j] = it;
}

// One lane per template: the SHA-256 state after the prefix's full 64-byte blocks (ECDSA's
// e = SHA-256(SignableData) resumes from it: 3 of the 5 compressions of a 269-byte message).
__global__ void __launch_bounds__(64) k_tmpl_mid(const cg_signable_tmpl* __restrict__ tmpls, uint32_t n_tmpls,
                                                 const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                 TmplMid* __restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tmpls) return;
  const cg_signable_tmpl tm = tmpls[t];
  TmplMid r;
  sha256_init(r.state);
  r.blocks = 0;
  r.pad[0] = r.pad[1] = r.pad[2] = 0;
  if (tmpl_ok(tm, arena_len)) {
    const uint64_t lr = round4(arena_len);
    for (uint32_t b = 0; b < tm.prefix_len / 64; ++b) {
      uint32_t w[16];
      for (int j = 0; j < 16; ++j) {
        uint32_t v = 0;
        for (int q = 0; q < 4; ++q) v = (v << 8) | (cg_ld_bytes4(arena, lr, tm.prefix_off + 64u * b + 4u * j + q) & 0xffu);
        w[j] = v;
      }
      sha256_compress(r.state, w);
      r.blocks = b + 1;
    }
  }
  out[t] = r;
}

__global__ void __launch_bounds__(256) k_splice(const cg_txsig* __restrict__ sigs, uint64_t n_sigs,
                                                const cg_signable_tmpl* __restrict__ tmpls, uint32_t n_tmpls,
                                                const uint8_t* __restrict__ tx_status, uint64_t n_tx,
                                                const uint8_t* __restrict__ ids, const uint8_t* __restrict__ arena,
                                                uint64_t arena_len, uint64_t head, uint64_t slot,
                                                uint8_t* __restrict__ msgs) {
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
  ((uint32_t*)(msgs + head))[g] = v;
}

uint64_t tx_msgs_head(uint32_t n_tmpls) { return tmpl_mid_bytes(n_tmpls); }

hipError_t launch_tx_sig_items(const cg_txsig* d_sigs, uint64_t n_sigs, const cg_signable_tmpl* d_tmpls,
                               uint32_t n_tmpls, const uint8_t* d_tx_status, uint64_t n_tx, const uint8_t* d_ids,
                               const uint8_t* d_arena, uint64_t arena_len, uint64_t slot, cg_item* d_items,
                               uint8_t* d_msgs, hipStream_t stream) {
  if (n_sigs == 0) return hipSuccess;
  const uint32_t B = 256;
  const uint64_t head = tmpl_mid_bytes(n_tmpls);
  if (n_tmpls)
    hipLaunchKernelGGL(k_tmpl_mid, dim3((n_tmpls + 63) / 64), dim3(64), 0, stream, d_tmpls, n_tmpls, d_arena,
                       arena_len, (TmplMid*)d_msgs);
  hipLaunchKernelGGL(k_txsig_items, dim3((unsigned)((n_sigs + B - 1) / B)), dim3(B), 0, stream, d_sigs, n_sigs,
                     d_tmpls, n_tmpls, d_tx_status, n_tx, arena_len, head, slot, d_items);
  const uint64_t words = n_sigs * (slot >> 2);
  hipLaunchKernelGGL(k_splice, dim3((unsigned)((words + B - 1) / B)), dim3(B), 0, stream, d_sigs, n_sigs, d_tmpls,
                     n_tmpls, d_tx_status, n_tx, d_ids, d_arena, arena_len, head, slot, d_msgs);
  return hipGetLastError();
}

}  // namespace cg
