// Transaction pipeline glue for gfx950: from device-computed WireTransaction ids to the
// per-signature verify items (cg_verify_transactions*, include/cordagpu.h).
//
//   k_txsig_items   one lane per signature: a cg_item whose clear data is the splice of its
//                   template and tx id (flags CG_ITEM_MSG_WS | TMPL | FUSED), or an out-of-range key
//                   index (-> CG_NOT_RUN) when its transaction has no id or its template /
//                   transaction index is invalid. tx_status == nullptr: the ids are the
//                   caller's (cg_verify_tx_signatures*), every one valid
//   k_tmpl_prep     one block per SignableData template: its image, SHA-256 midstate and the
//                   Ed25519 challenge's block-1 schedule (keyws.h TmplW512); the
//                   hash kernels read SignableData(id, metadata).serialize() (Crypto.kt:499-502)
//                   = prefix || id || suffix straight from the image and the id (SpliceLd)
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
                                                     uint64_t arena_len, cg_item* __restrict__ items) {
  front_prio();
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
    it.msg_off = s.tx_idx;  // fused: the hash kernels read the splice (keyws.h item_splice)
    it.msg_len = t.prefix_len + 32u + t.suffix_len;
    it.key_idx = s.key_idx;
    it.reserved0 = CG_ITEM_MSG_WS | CG_ITEM_TMPL | CG_ITEM_FUSED;
    it.reserved1 = s.tmpl;
  } else {
    it.msg_off = 0;
    it.msg_len = 0;
    it.key_idx = 0xffffffffu;  // k_misc_status: CG_NOT_RUN
    it.reserved0 = 0;
  }
  items[j] = it;
}

// ---- the 12-byte signature table (cg_txsig_packed, include/cordagpu.h): signature j's bytes start at
// the sum of round_up(sig_len, 4) over the records before it, in the caller's dense signature stream
#define SIG12_BLOCK 256
__device__ __forceinline__ uint32_t sig12_span(uint32_t len) { return (len + 3u) & ~3u; }

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = (int)(threadIdx.x & 63);
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(v, d, 64);
    if (lane >= d) v += u;
  }
  return v;
}

// sums[b] = the stream bytes of records [first + 256 b, first + 256 (b + 1)) ∩ [first, first + n)
__global__ void __launch_bounds__(SIG12_BLOCK) k_sig12_blocksum(const cg_txsig_packed* __restrict__ sigs,
                                                                uint64_t first, uint64_t n, uint64_t* __restrict__ sums) {
  const uint64_t j = (uint64_t)blockIdx.x * SIG12_BLOCK + threadIdx.x;
  uint32_t v = j < n ? sig12_span(sigs[first + j].sig_len) : 0u;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  __shared__ uint32_t part[SIG12_BLOCK / 64];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int w = 0; w < SIG12_BLOCK / 64; ++w) t += part[w];
    sums[blockIdx.x] = t;
  }
}

// sums[0 .. nb) -> base + their exclusive prefix sums, in place (one block)
__global__ void __launch_bounds__(1024) k_sig12_scan(uint64_t* __restrict__ sums, uint64_t nb, uint64_t base) {
  __shared__ uint64_t sh[1024];
  const uint32_t t = threadIdx.x;
  const uint64_t per = (nb + 1023) / 1024, lo = t * per, hi = lo + per < nb ? lo + per : nb;
  uint64_t s = 0;
  for (uint64_t i = lo; i < hi; ++i) s += sums[i];
  sh[t] = s;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    const uint64_t u = t >= d ? sh[t - d] : 0;
    __syncthreads();
    sh[t] += u;
    __syncthreads();
  }
  uint64_t run = base + sh[t] - s;
  for (uint64_t i = lo; i < hi; ++i) {
    const uint64_t x = sums[i];
    sums[i] = run;
    run += x;
  }
}

// k_txsig_items over the 12-byte table: block b's records start at stream offset bases[b]; each
// lane's offset is that plus the block's exclusive scan of the spans before it
__global__ void __launch_bounds__(SIG12_BLOCK) k_txsig12_items(const cg_txsig_packed* __restrict__ sigs, uint64_t first,
                                                               uint64_t n_sigs, const uint64_t* __restrict__ bases,
                                                               uint64_t sig_region, uint64_t sig_bytes_len,
                                                               const cg_signable_tmpl* __restrict__ tmpls,
                                                               uint32_t n_tmpls, uint64_t n_tx, uint64_t arena_len,
                                                               cg_item* __restrict__ items) {
  front_prio();
  const uint64_t jj = (uint64_t)blockIdx.x * SIG12_BLOCK + threadIdx.x;
  const bool live = jj < n_sigs;
  cg_txsig_packed s = {0, 0, 0, 0};
  if (live) s = sigs[first + jj];
  const uint32_t span = live ? sig12_span(s.sig_len) : 0u;
  const uint32_t incl = wave_incl_scan(span);
  __shared__ uint32_t wtot[SIG12_BLOCK / 64];
  if ((threadIdx.x & 63) == 63) wtot[threadIdx.x >> 6] = incl;
  __syncthreads();
  uint32_t wbase = 0;
  for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) wbase += wtot[w];
  if (!live) return;
  cg_item it;
  const uint64_t so = bases[blockIdx.x] + (wbase + incl - span);  // offset in the signature stream
  it.sig_off = sig_region + so;
  it.sig_len = s.sig_len;
  it.reserved1 = 0;
  bool ok = s.tx_idx < n_tx && s.tmpl < n_tmpls && so <= sig_bytes_len && s.sig_len <= sig_bytes_len - so;
  cg_signable_tmpl t = {0, 0, 0, 0};
  if (ok) {
    t = tmpls[s.tmpl];
    ok = tmpl_ok(t, arena_len);
  }
  if (ok) {
    it.msg_off = s.tx_idx;  // fused: the hash kernels read the splice (keyws.h item_splice)
    it.msg_len = t.prefix_len + 32u + t.suffix_len;
    it.key_idx = s.key_idx;
    it.reserved0 = CG_ITEM_MSG_WS | CG_ITEM_TMPL | CG_ITEM_FUSED;
    it.reserved1 = s.tmpl;
  } else {
    it.msg_off = 0;
    it.msg_len = 0;
    it.key_idx = 0xffffffffu;  // k_misc_status: CG_NOT_RUN
    it.reserved0 = 0;
  }
  items[first + jj] = it;
}

size_t tx_sig12_scratch_bytes(uint64_t n) { return 8 * ((n + SIG12_BLOCK - 1) / SIG12_BLOCK + 1); }

hipError_t launch_tx_sig12_bases(const cg_txsig_packed* d_sigs, uint64_t first, uint64_t n, uint64_t base,
                                 uint64_t* d_bases, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint64_t nb = (n + SIG12_BLOCK - 1) / SIG12_BLOCK;
  hipLaunchKernelGGL(k_sig12_blocksum, dim3((unsigned)nb), dim3(SIG12_BLOCK), 0, stream, d_sigs, first, n, d_bases);
  hipLaunchKernelGGL(k_sig12_scan, dim3(1), dim3(1024), 0, stream, d_bases, nb, base);
  return hipGetLastError();
}

hipError_t launch_tx_sig12_range(const cg_txsig_packed* d_sigs, uint64_t first, uint64_t n, uint64_t sig_region,
                                 uint64_t sig_bytes_len, uint64_t base, const uint64_t* d_bases,
                                 const cg_signable_tmpl* d_tmpls,
                                 uint32_t n_tmpls, uint64_t n_tx, uint64_t arena_len, cg_item* d_items,
                                 void* d_scratch, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint64_t* bases = d_bases ? d_bases + first / SIG12_BLOCK : (const uint64_t*)d_scratch;
  if (d_bases && first % SIG12_BLOCK) return hipErrorInvalidValue;  // precomputed bases are per aligned block
  if (!d_bases) {
    const hipError_t e = launch_tx_sig12_bases(d_sigs, first, n, base, (uint64_t*)d_scratch, stream);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_txsig12_items, dim3((unsigned)((n + SIG12_BLOCK - 1) / SIG12_BLOCK)), dim3(SIG12_BLOCK), 0,
                     stream, d_sigs, first, n, bases, sig_region, sig_bytes_len, d_tmpls, n_tmpls, n_tx, arena_len,
                     d_items);
  return hipGetLastError();
}

// The message workspace (keyws.h SpliceHdr): the header, per template its SHA-256 midstate record
// (ECDSA's e = SHA-256(M) resumes after the prefix's full 64-byte blocks: 3 of the 5 compressions of
// a 269-byte message) and its image prefix || 0^32 || suffix, zero-padded to the slot; the hash
// kernels OR each signature's id into the image as they read it (SpliceLd), so no message is written.
static __host__ __device__ inline uint64_t tx_img_off(uint32_t n_tmpls) { return tmpl_mid_bytes(n_tmpls); }
uint64_t tx_msgs_head(uint32_t n_tmpls, uint64_t slot) {
  return (tx_img_off(n_tmpls) + (uint64_t)n_tmpls * slot + 255) & ~(uint64_t)255;
}

// One block of 64 lanes per template: the image words lane-strided, the midstate on lane 0.
__global__ void __launch_bounds__(64) k_tmpl_prep(const cg_signable_tmpl* __restrict__ tmpls, uint32_t n_tmpls,
                                                  const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                  uint64_t slot, const uint8_t* __restrict__ ids, uint64_t n_ids,
                                                  uint8_t* __restrict__ msgs) {
  const uint32_t t = blockIdx.x;
  if (t == 0 && threadIdx.x == 0) {
    SpliceHdr h;
    h.ids = (uint64_t)(uintptr_t)ids;
    h.n_ids = n_ids;
    h.img_off = tx_img_off(n_tmpls);
    h.slot = slot;
    h.w512_off = tmpl_w512_off(n_tmpls);
    *(SpliceHdr*)msgs = h;
  }
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
  const bool ed_mid = ok && tm.prefix_len >= TMPL_ED_MID_MIN_PREFIX;
  if (threadIdx.x == 1) {  // the Ed25519 challenge's block 1 = message bytes 64..191 (keyws.h TmplW512)
    uint64_t* wk = ((TmplW512*)(msgs + tmpl_w512_off(n_tmpls)) + t)->wk;
    uint64_t w[16];
    for (int j = 0; j < 16; ++j) {
      uint64_t v = 0;
      for (int q = 0; q < 8; ++q) v = (v << 8) | (ed_mid ? byte_at(64ull + 8u * j + q) : 0u);
      w[j] = v;
      wk[j] = v + cg_k512(j);
    }
    for (int r = 16; r < 80; r += 16)
      for (int j = 0; j < 16; ++j) wk[r + j] = sha512_sched(w, j) + cg_k512(r + j);
  }
  if (threadIdx.x != 0) return;
  TmplMid r;
  sha256_init(r.state);
  r.blocks = 0;
  r.prefix_len = tm.prefix_len;
  r.ed_mid = ed_mid ? 1u : 0u;
  r.pad = 0;
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
  ((TmplMid*)(msgs + SPLICE_HDR_BYTES))[t] = r;
}

hipError_t launch_tx_sig_templates(const cg_signable_tmpl* d_tmpls, uint32_t n_tmpls, const uint8_t* d_arena,
                                   uint64_t arena_len, uint64_t slot, const uint8_t* d_ids, uint64_t n_ids,
                                   uint8_t* d_msgs, hipStream_t stream) {
  hipLaunchKernelGGL(k_tmpl_prep, dim3(n_tmpls ? n_tmpls : 1), dim3(64), 0, stream, d_tmpls, n_tmpls, d_arena,
                     arena_len, slot, d_ids, n_ids, d_msgs);
  return hipGetLastError();
}

hipError_t launch_tx_sig_range(const cg_txsig* d_sigs, uint64_t first, uint64_t n, const cg_signable_tmpl* d_tmpls,
                               uint32_t n_tmpls, const uint8_t* d_tx_status, uint64_t n_tx, const uint8_t* d_ids,
                               uint64_t arena_len, uint64_t slot, cg_item* d_items, uint8_t* d_msgs,
                               hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint32_t B = 256;
  (void)d_ids;
  (void)slot;
  (void)d_msgs;
  hipLaunchKernelGGL(k_txsig_items, dim3((unsigned)((n + B - 1) / B)), dim3(B), 0, stream, d_sigs, first, n, d_tmpls,
                     n_tmpls, d_tx_status, n_tx, arena_len, d_items);
  return hipGetLastError();
}

hipError_t launch_tx_sig_items(const cg_txsig* d_sigs, uint64_t n_sigs, const cg_signable_tmpl* d_tmpls,
                               uint32_t n_tmpls, const uint8_t* d_tx_status, uint64_t n_tx, const uint8_t* d_ids,
                               const uint8_t* d_arena, uint64_t arena_len, uint64_t slot, cg_item* d_items,
                               uint8_t* d_msgs, hipStream_t stream) {
  if (n_sigs == 0) return hipSuccess;
  hipError_t e = launch_tx_sig_templates(d_tmpls, n_tmpls, d_arena, arena_len, slot, d_ids, n_tx, d_msgs, stream);
  if (e == hipSuccess)
    e = launch_tx_sig_range(d_sigs, 0, n_sigs, d_tmpls, n_tmpls, d_tx_status, n_tx, d_ids, arena_len, slot, d_items,
                            d_msgs, stream);
  return e;
}

}  // namespace cg
