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

__global__ void __launch_bounds__(256) k_txsig_items(const cg_txsig* __restrict__ sigs, uint64_t first, uint64_t n_sigs,
                                                     const cg_signable_tmpl* __restrict__ tmpls, uint32_t n_tmpls,
                                                     const uint8_t* __restrict__ tx_status, uint64_t n_tx,
                                                     uint64_t arena_len, uint64_t head, uint64_t slot,
                                                     cg_item* __restrict__ items) {
  const uint64_t j = first + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= first + n_sigs) return;
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

// The message workspace's head: per template its SHA-256 midstate record (ECDSA's e = SHA-256(M)
// resumes after the prefix's full 64-byte blocks: 3 of the 5 compressions of a 269-byte message),
// then its image prefix || 0^32 || suffix, zero-padded to the slot (k_splice ORs the id into it).
static __host__ __device__ inline uint64_t tx_img_off(uint32_t n_tmpls) { return tmpl_mid_bytes(n_tmpls); }
uint64_t tx_msgs_head(uint32_t n_tmpls, uint64_t slot) {
  return (tx_img_off(n_tmpls) + (uint64_t)n_tmpls * slot + 255) & ~(uint64_t)255;
}

// One block of 64 lanes per template: the image words lane-strided, the midstate on lane 0.
__global__ void __launch_bounds__(64) k_tmpl_prep(const cg_signable_tmpl* __restrict__ tmpls, uint32_t n_tmpls,
                                                  const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                  uint64_t slot, uint8_t* __restrict__ msgs) {
  const uint32_t t = blockIdx.x;
  if (t >= n_tmpls) return;
  const cg_signable_tmpl tm = tmpls[t];
  const bool ok = tmpl_ok(tm, arena_len);
  const uint64_t lr = round4(arena_len);
  auto byte_at = [&](uint64_t x) -> uint32_t {  // template byte x (id bytes read as 0)
    if (!ok) return 0u;
    if (x < tm.prefix_len) return cg_ld_bytes4(arena, lr, tm.prefix_off + x) & 0xffu;
    if (x < tm.prefix_len + 32u) return 0u;
    if (x < (uint64_t)tm.prefix_len + 32u + tm.suffix_len)
      return cg_ld_bytes4(arena, lr, tm.suffix_off + (x - tm.prefix_len - 32u)) & 0xffu;
    return 0u;
  };
  uint32_t* img = (uint32_t*)(msgs + tx_img_off(n_tmpls) + (uint64_t)t * slot);
  for (uint32_t w = threadIdx.x; w < slot / 4; w += 64) {
    uint32_t v = 0;
    for (int q = 0; q < 4; ++q) v |= byte_at(4ull * w + q) << (8 * q);
    img[w] = v;
  }
  if (threadIdx.x != 0) return;
  TmplMid r;
  sha256_init(r.state);
  r.blocks = 0;
  r.pad[0] = r.pad[1] = r.pad[2] = 0;
  if (ok) {
    for (uint32_t b = 0; b < tm.prefix_len / 64; ++b) {
      uint32_t w[16];
      for (int j = 0; j < 16; ++j) {
        uint32_t v = 0;
        for (int q = 0; q < 4; ++q) v = (v << 8) | byte_at(64ull * b + 4u * j + q);
        w[j] = v;
      }
      sha256_compress(r.state, w);
      r.blocks = b + 1;
    }
  }
  ((TmplMid*)msgs)[t] = r;
}

// One lane per 16-byte chunk of a signature's message slot: the template image's chunk with the
// signature's tx id ORed in where the chunk overlaps it (two aligned id dwords and a funnel shift
// per overlapping word); coalesced 16-byte stores. SignableData(id, metadata).serialize() =
// prefix || id || suffix (Crypto.kt:499-502).
__global__ void __launch_bounds__(256) k_splice(const cg_txsig* __restrict__ sigs, uint64_t first, uint64_t n_sigs,
                                                const cg_signable_tmpl* __restrict__ tmpls, uint32_t n_tmpls,
                                                const uint8_t* __restrict__ tx_status, uint64_t n_tx,
                                                const uint8_t* __restrict__ ids, uint64_t arena_len, uint64_t head,
                                                uint64_t slot, uint8_t* __restrict__ msgs) {
  const uint64_t cps = slot >> 4;
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t jl = g / cps, c = g % cps;
  if (jl >= n_sigs) return;
  const uint64_t j = first + jl;
  const cg_txsig s = sigs[j];
  uint4 v = make_uint4(0, 0, 0, 0);
  if (s.tx_idx < n_tx && s.tmpl < n_tmpls && (!tx_status || tx_status[s.tx_idx] == 0)) {
    const cg_signable_tmpl t = tmpls[s.tmpl];
    if (tmpl_ok(t, arena_len)) {
      v = *(const uint4*)(msgs + tx_img_off(n_tmpls) + (uint64_t)s.tmpl * slot + 16 * c);
      const int64_t x0 = (int64_t)(16 * c) - (int64_t)t.prefix_len;  // id byte at the chunk's start
      if (x0 > -16 && x0 < 32) {
        const uint32_t* id = (const uint32_t*)(ids + 32ull * s.tx_idx);
        uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t x = x0 + 4 * q;
          if (x <= -4 || x >= 32) continue;
          const int64_t a = x >= 0 ? x >> 2 : -1;
          const uint32_t r = (uint32_t)(x - 4 * a);
          const uint32_t lo = a >= 0 ? id[a] : 0u;
          const uint32_t hi = a + 1 < 8 ? id[a + 1] : 0u;
          wv[q] |= r ? (lo >> (8 * r)) | (hi << (32 - 8 * r)) : lo;
        }
        v = make_uint4(wv[0], wv[1], wv[2], wv[3]);
      }
    }
  }
  *(uint4*)(msgs + head + j * slot + 16 * c) = v;
}

hipError_t launch_tx_sig_templates(const cg_signable_tmpl* d_tmpls, uint32_t n_tmpls, const uint8_t* d_arena,
                                   uint64_t arena_len, uint64_t slot, uint8_t* d_msgs, hipStream_t stream) {
  if (n_tmpls)
    hipLaunchKernelGGL(k_tmpl_prep, dim3(n_tmpls), dim3(64), 0, stream, d_tmpls, n_tmpls, d_arena, arena_len, slot,
                       d_msgs);
  return hipGetLastError();
}

hipError_t launch_tx_sig_range(const cg_txsig* d_sigs, uint64_t first, uint64_t n, const cg_signable_tmpl* d_tmpls,
                               uint32_t n_tmpls, const uint8_t* d_tx_status, uint64_t n_tx, const uint8_t* d_ids,
                               uint64_t arena_len, uint64_t slot, cg_item* d_items, uint8_t* d_msgs,
                               hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint32_t B = 256;
  const uint64_t head = tx_msgs_head(n_tmpls, slot);
  hipLaunchKernelGGL(k_txsig_items, dim3((unsigned)((n + B - 1) / B)), dim3(B), 0, stream, d_sigs, first, n, d_tmpls,
                     n_tmpls, d_tx_status, n_tx, arena_len, head, slot, d_items);
  const uint64_t chunks = n * (slot >> 4);
  hipLaunchKernelGGL(k_splice, dim3((unsigned)((chunks + B - 1) / B)), dim3(B), 0, stream, d_sigs, first, n, d_tmpls,
                     n_tmpls, d_tx_status, n_tx, d_ids, arena_len, head, slot, d_msgs);
  return hipGetLastError();
}

hipError_t launch_tx_sig_items(const cg_txsig* d_sigs, uint64_t n_sigs, const cg_signable_tmpl* d_tmpls,
                               uint32_t n_tmpls, const uint8_t* d_tx_status, uint64_t n_tx, const uint8_t* d_ids,
                               const uint8_t* d_arena, uint64_t arena_len, uint64_t slot, cg_item* d_items,
                               uint8_t* d_msgs, hipStream_t stream) {
  if (n_sigs == 0) return hipSuccess;
  hipError_t e = launch_tx_sig_templates(d_tmpls, n_tmpls, d_arena, arena_len, slot, d_msgs, stream);
  if (e == hipSuccess)
    e = launch_tx_sig_range(d_sigs, 0, n_sigs, d_tmpls, n_tmpls, d_tx_status, n_tx, d_ids, arena_len, slot, d_items,
                            d_msgs, stream);
  return e;
}

}  // namespace cg
