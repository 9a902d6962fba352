// Batch signature verification kernels for gfx950.
//
// Pipeline per batch (all on the caller's stream, no host round trip):
//   k_ed_keyprep   one lane per distinct key: decode A, canonical Abyte, 8 multiples of -A
//   k_ed_verify    one lane per Ed25519 item: SHA-512 challenge, scalar prep, 64-window
//                  double-scalar multiplication, encode + byte compare
//   k_misc_status  one lane per item of an unsupported scheme / bad key index
// Replaces, per item, the JCA call at core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:553-559
// behind Crypto.doVerify (Crypto.kt:474-484).
#include <hip/hip_runtime.h>

#include "ecdsa.h"
#include "ed25519.h"
#include "engine.h"

namespace cg {

__constant__ Ed25519Consts c_ed;

static const uint8_t ED_SPKI_PREFIX[12] = {0x30, 0x2a, 0x30, 0x05, 0x06, 0x03, 0x2b, 0x65, 0x70, 0x03, 0x21, 0x00};

__device__ __forceinline__ uint64_t round4(uint64_t x) { return (x + 3) & ~(uint64_t)3; }

__device__ __forceinline__ bool in_arena(uint64_t off, uint64_t len, uint64_t arena_len) {
  return off <= arena_len && len <= arena_len - off;
}

__global__ void __launch_bounds__(256) k_ed_keyprep(const cg_key* __restrict__ keys, uint32_t n_keys,
                                                    const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                    EdKeyPrep* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_keys) return;
  const cg_key k = keys[i];
  if (k.scheme != CG_EDDSA_ED25519_SHA512) return;
  EdKeyPrep& kp = out[i];
  const uint64_t lr = round4(arena_len);
  uint64_t a_off = k.off;
  bool ok = in_arena(k.off, k.len, arena_len);
  if (ok && k.fmt == CG_KEY_RAW) {
    ok = k.len == 32;
  } else if (ok && k.fmt == CG_KEY_SPKI) {
    ok = k.len == 44;
    for (int b = 0; ok && b < 12; ++b) ok = (cg_ld_bytes4(arena, lr, k.off + b) & 0xffu) == ED_SPKI_PREFIX[b];
    a_off = k.off + 12;
  } else {
    ok = false;
  }
  if (!ok) {
    kp.status = CG_KEY_INVALID;
    return;
  }
  uint32_t aw[8];
#pragma unroll
  for (int w = 0; w < 8; ++w) aw[w] = cg_ld_bytes4(arena, lr, a_off + 4 * w);
  EdKeyPrep local;
  ed_key_prep(local, aw, c_ed);
  kp = local;
  if (local.status != ED_ST_VALID) kp.status = CG_KEY_INVALID;
}

__global__ void __launch_bounds__(256) k_ed_verify(const cg_item* __restrict__ items, uint64_t n_items,
                                                   const cg_key* __restrict__ keys, uint32_t n_keys,
                                                   const EdKeyPrep* __restrict__ kps,
                                                   const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                   uint32_t mode, uint8_t* __restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_items) return;
  const cg_item it = items[i];
  if (it.key_idx >= n_keys) return;
  const cg_key k = keys[it.key_idx];
  if (k.scheme != CG_EDDSA_ED25519_SHA512) return;
  const EdKeyPrep* kp = kps + it.key_idx;
  uint8_t st;
  if (kp->status != 0) {
    st = CG_KEY_INVALID;
  } else if (mode == CG_MODE_DOVERIFY && (it.sig_len == 0 || it.msg_len == 0)) {
    st = CG_EMPTY;
  } else if (!in_arena(it.sig_off, it.sig_len, arena_len) || !in_arena(it.msg_off, it.msg_len, arena_len)) {
    st = CG_NOT_RUN;
  } else if (it.sig_len != 64) {
    st = CG_SIG_MALFORMED;
  } else {
    const uint64_t lr = round4(arena_len);
    uint32_t sw[16];
#pragma unroll
    for (int w = 0; w < 16; ++w) sw[w] = cg_ld_bytes4(arena, lr, it.sig_off + 4 * w);
    st = (uint8_t)ed_verify_core(*kp, kp->tab, sw, arena, lr, it.msg_off, it.msg_len, c_ed, c_ed.Btab);
  }
  status[i] = st;
}

// ------------------------------------------------------------------ ECDSA (BC 1.57 semantics)
__constant__ EcConsts c_ec[2];  // [CG_CURVE_K1], [CG_CURVE_R1]

template <int C>
__global__ void __launch_bounds__(64) k_ec_keyprep(const cg_key* __restrict__ keys, uint32_t n_keys,
                                                   const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                   EcKeyPrep* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_keys) return;
  const cg_key k = keys[i];
  const uint8_t want = C == CG_CURVE_R1 ? CG_ECDSA_SECP256R1_SHA256 : CG_ECDSA_SECP256K1_SHA256;
  if (k.scheme != want) return;
  if (!in_arena(k.off, k.len, arena_len)) {
    out[i].status = CG_KEY_INVALID;
    return;
  }
  const uint32_t st = ec_key_prep_bytes<C>(out[i], arena, round4(arena_len), k.off, k.len, k.fmt, c_ec[C]);
  out[i].status = st ? CG_KEY_INVALID : 0u;
}

template <int C>
__global__ void __launch_bounds__(256) k_ec_verify(const cg_item* __restrict__ items, uint64_t n_items,
                                                   const cg_key* __restrict__ keys, uint32_t n_keys,
                                                   const EcKeyPrep* __restrict__ kps,
                                                   const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                   uint32_t mode, uint8_t* __restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_items) return;
  const cg_item it = items[i];
  if (it.key_idx >= n_keys) return;
  const uint8_t want = C == CG_CURVE_R1 ? CG_ECDSA_SECP256R1_SHA256 : CG_ECDSA_SECP256K1_SHA256;
  if (keys[it.key_idx].scheme != want) return;
  const EcKeyPrep* kp = kps + it.key_idx;
  uint8_t st;
  if (kp->status != 0) {
    st = CG_KEY_INVALID;
  } else if (mode == CG_MODE_DOVERIFY && (it.sig_len == 0 || it.msg_len == 0)) {
    st = CG_EMPTY;
  } else if (!in_arena(it.sig_off, it.sig_len, arena_len) || !in_arena(it.msg_off, it.msg_len, arena_len)) {
    st = CG_NOT_RUN;
  } else {
    st = (uint8_t)ecdsa_verify_core<C>(*kp, arena, round4(arena_len), it.sig_off, it.sig_len, it.msg_off, it.msg_len,
                                       c_ec[C]);
  }
  status[i] = st;
}

__global__ void k_misc_status(const cg_item* __restrict__ items, uint64_t n_items, const cg_key* __restrict__ keys,
                              uint32_t n_keys, uint8_t* __restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_items) return;
  const uint32_t ki = items[i].key_idx;
  if (ki >= n_keys) {
    status[i] = CG_NOT_RUN;
    return;
  }
  const uint8_t s = keys[ki].scheme;
  if (s != CG_EDDSA_ED25519_SHA512 && s != CG_ECDSA_SECP256R1_SHA256 && s != CG_ECDSA_SECP256K1_SHA256)
    status[i] = CG_UNSUPPORTED;
}

hipError_t upload_constants() {
  Ed25519Consts h;
  ed_consts_init(h);
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_ed), &h, sizeof h, 0, hipMemcpyHostToDevice);
  if (e != hipSuccess) return e;
  EcConsts k[2];
  ec_consts_init<CG_CURVE_K1>(k[CG_CURVE_K1]);
  ec_consts_init<CG_CURVE_R1>(k[CG_CURVE_R1]);
  return hipMemcpyToSymbol(HIP_SYMBOL(c_ec), k, sizeof k, 0, hipMemcpyHostToDevice);
}

// workspace: [EdKeyPrep x n_keys][EcKeyPrep x n_keys]
static size_t ed_region(uint32_t n_keys) { return ((size_t)(n_keys ? n_keys : 1) * sizeof(EdKeyPrep) + 255) & ~(size_t)255; }
size_t keyprep_bytes(uint32_t n_keys) { return ed_region(n_keys) + (size_t)(n_keys ? n_keys : 1) * sizeof(EcKeyPrep); }

hipError_t launch_keyprep(const cg_key* d_keys, uint32_t n_keys, const uint8_t* d_arena, uint64_t arena_len,
                          void* d_keyprep, hipStream_t stream) {
  if (n_keys == 0) return hipSuccess;
  const uint32_t B = 64;  // one wave per block: keys are few, spread them over CUs
  const dim3 g((n_keys + B - 1) / B);
  EcKeyPrep* ec = (EcKeyPrep*)((uint8_t*)d_keyprep + ed_region(n_keys));
  hipLaunchKernelGGL(k_ed_keyprep, g, dim3(B), 0, stream, d_keys, n_keys, d_arena, arena_len, (EdKeyPrep*)d_keyprep);
  hipLaunchKernelGGL(k_ec_keyprep<CG_CURVE_R1>, g, dim3(B), 0, stream, d_keys, n_keys, d_arena, arena_len, ec);
  hipLaunchKernelGGL(k_ec_keyprep<CG_CURVE_K1>, g, dim3(B), 0, stream, d_keys, n_keys, d_arena, arena_len, ec);
  return hipGetLastError();
}

hipError_t launch_items(const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                        const uint8_t* d_arena, uint64_t arena_len, uint32_t mode, uint8_t* d_status,
                        const void* d_keyprep, hipStream_t stream) {
  if (n_items == 0) return hipSuccess;
  const uint32_t B = 256;
  const uint64_t grid = (n_items + B - 1) / B;
  hipLaunchKernelGGL(k_misc_status, dim3((unsigned)grid), dim3(B), 0, stream, d_items, n_items, d_keys, n_keys,
                     d_status);
  hipLaunchKernelGGL(k_ed_verify, dim3((unsigned)grid), dim3(B), 0, stream, d_items, n_items, d_keys, n_keys,
                     (const EdKeyPrep*)d_keyprep, d_arena, arena_len, mode, d_status);
  const EcKeyPrep* ec = (const EcKeyPrep*)((const uint8_t*)d_keyprep + ed_region(n_keys));
  hipLaunchKernelGGL(k_ec_verify<CG_CURVE_R1>, dim3((unsigned)grid), dim3(B), 0, stream, d_items, n_items, d_keys,
                     n_keys, ec, d_arena, arena_len, mode, d_status);
  hipLaunchKernelGGL(k_ec_verify<CG_CURVE_K1>, dim3((unsigned)grid), dim3(B), 0, stream, d_items, n_items, d_keys,
                     n_keys, ec, d_arena, arena_len, mode, d_status);
  return hipGetLastError();
}

hipError_t launch_verify(const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                         const uint8_t* d_arena, uint64_t arena_len, uint32_t mode, uint8_t* d_status,
                         void* d_keyprep, hipStream_t stream) {
  if (n_items == 0) return hipSuccess;
  hipError_t e = launch_keyprep(d_keys, n_keys, d_arena, arena_len, d_keyprep, stream);
  if (e != hipSuccess) return e;
  return launch_items(d_keys, n_keys, d_items, n_items, d_arena, arena_len, mode, d_status, d_keyprep, stream);
}

}  // namespace cg
