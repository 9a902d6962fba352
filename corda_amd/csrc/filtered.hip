// Tear-off verification for gfx950: FilteredTransaction.verify / PartialMerkleTree.verify
// (SURVEY §8 f4), the non-validating notary's per-transaction check.
//
//   k_ftx_leaves  one lane per visible component: serializedHash(x, nonce) = SHA256(blob || nonce)
//                 (MerkleTransaction.kt:23-28,137); a salt component hashes without the nonce;
//                 CG_FLEAF_HASH passes a precomputed hash through (PartialMerkleTree.verify)
//   k_ftx_verify  one lane per filtered transaction: the empty check (MerkleTransaction.kt:173-178),
//                 the partial tree reduced bottom-up from its post-order stream with a hash
//                 stack (PartialMerkleTree.kt:143-156: IncludedLeaf / Leaf push their hash,
//                 Node = hashConcat(left, right)), the used-hash multiset compared with the leaf
//                 hashes (PartialMerkleTree.kt:134: groupBy equality == multiset equality) and
//                 the root compared with rootHash (:136)
//
// The JVM walks the tree recursively; a post-order stream plus an explicit stack is the same
// reduction without recursion. The stack lives in the lane's scratch (CG_PMT_MAX_DEPTH x 32 B):
// honest trees from PartialMerkleTree.build are at most log2(leaves) + 1 deep.
#include <hip/hip_runtime.h>

#include "engine.h"
#include "sha2.h"

namespace cg {

__device__ __forceinline__ uint64_t ftx_r4(uint64_t x) { return (x + 3) & ~(uint64_t)3; }

__device__ __forceinline__ bool in_arena(uint64_t off, uint64_t len, uint64_t arena_len) {
  return off <= arena_len && len <= arena_len - off;
}

// 32-byte hash at arena[off] as 8 big-endian words
__device__ __forceinline__ void ld_hash_be(uint32_t v[8], const uint8_t* arena, uint64_t lr, uint64_t off) {
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = __builtin_bswap32(cg_ld_bytes4(arena, lr, off + 4 * k));
}

// SHA-256 of the 64-byte message left || right (SecureHash.hashConcat, SecureHash.kt:25)
__device__ __forceinline__ void hash_concat_be(uint32_t out[8], const uint32_t l[8], const uint32_t r[8]) {
  uint32_t s[8], w[16];
  sha256_init(s);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    w[k] = l[k];
    w[8 + k] = r[k];
  }
  sha256_compress(s, w);
  w[0] = 0x80000000u;
#pragma unroll
  for (int k = 1; k < 15; ++k) w[k] = 0;
  w[15] = 512;
  sha256_compress(s, w);
#pragma unroll
  for (int k = 0; k < 8; ++k) out[k] = s[k];
}

// Leaf hashes: ws_hash[32 * i] (big-endian words), ws_bad[i] = 1 if the leaf is outside the arena.
__global__ void __launch_bounds__(256) k_ftx_leaves(const cg_filtered_leaf* __restrict__ leaves, uint64_t n_leaves,
                                                    const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                    uint32_t* __restrict__ ws_hash, uint8_t* __restrict__ ws_bad) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_leaves) return;
  const cg_filtered_leaf lf = leaves[i];
  const uint64_t lr = ftx_r4(arena_len);
  uint32_t h[8];
  bool bad = !in_arena(lf.off, lf.len, arena_len) || (lf.flags & ~(CG_FLEAF_SALT | CG_FLEAF_HASH)) != 0;
  if (!bad && (lf.flags & CG_FLEAF_HASH)) {
    bad = lf.len != 32;
    if (!bad) ld_hash_be(h, arena, lr, lf.off);
  } else if (!bad && (lf.flags & CG_FLEAF_SALT)) {
    sha256_arena_suffix(h, arena, lr, lf.off, lf.len, nullptr);
  } else if (!bad) {
    bad = !in_arena(lf.nonce_off, 32, arena_len);
    if (!bad) {
      uint32_t nonce[8];
      ld_hash_be(nonce, arena, lr, lf.nonce_off);
      sha256_arena_suffix(h, arena, lr, lf.off, lf.len, nonce);
    }
  }
  if (bad) {
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = 0;
  }
  uint4* o = (uint4*)(ws_hash + 8 * i);
  o[0] = make_uint4(h[0], h[1], h[2], h[3]);
  o[1] = make_uint4(h[4], h[5], h[6], h[7]);
  ws_bad[i] = bad ? 1 : 0;
}

__device__ __forceinline__ bool eq8(const uint32_t a[8], const uint32_t b[8]) {
  uint32_t d = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) d |= a[k] ^ b[k];
  return d == 0;
}

__device__ __forceinline__ void ld_ws(uint32_t v[8], const uint32_t* ws_hash, uint64_t i) {
  const uint4* p = (const uint4*)(ws_hash + 8 * i);
  const uint4 a = p[0], b = p[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

__global__ void __launch_bounds__(64) k_ftx_verify(const cg_filtered_tx* __restrict__ ftxs, uint64_t n_ftx,
                                                   const cg_pmt_node* __restrict__ nodes, uint64_t n_nodes,
                                                   uint64_t n_leaves, const uint8_t* __restrict__ arena,
                                                   uint64_t arena_len, const uint32_t* __restrict__ ws_hash,
                                                   const uint8_t* __restrict__ ws_bad, uint8_t* __restrict__ status) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_ftx) return;
  const cg_filtered_tx f = ftxs[t];
  const uint64_t lr = ftx_r4(arena_len);
  // table ranges and the root: malformed (3) if any lies outside
  if (f.n_nodes == 0 || f.first_node > n_nodes || f.n_nodes > n_nodes - f.first_node || f.first_leaf > n_leaves ||
      f.n_leaves > n_leaves - f.first_leaf || !in_arena(f.root_off, 32, arena_len) ||
      (f.flags & ~CG_FTX_FILTERED) != 0) {
    status[t] = 3;
    return;
  }
  for (uint32_t i = 0; i < f.n_leaves; ++i) {
    if (ws_bad[f.first_leaf + i]) {
      status[t] = 3;
      return;
    }
  }
  // FilteredTransaction.verify: no visible components -> MerkleTreeException
  if ((f.flags & CG_FTX_FILTERED) && f.n_leaves == 0) {
    status[t] = 2;
    return;
  }
  // post-order reduction of the partial tree
  uint32_t stk[CG_PMT_MAX_DEPTH][8];
  uint32_t sp = 0, used = 0;
  for (uint32_t j = 0; j < f.n_nodes; ++j) {
    const cg_pmt_node nd = nodes[f.first_node + j];
    if (nd.kind == CG_PMT_NODE) {
      if (sp < 2) {
        status[t] = 3;
        return;
      }
      uint32_t o[8];
      hash_concat_be(o, stk[sp - 2], stk[sp - 1]);
      sp -= 1;
#pragma unroll
      for (int k = 0; k < 8; ++k) stk[sp - 1][k] = o[k];
    } else if (nd.kind == CG_PMT_LEAF || nd.kind == CG_PMT_INCLUDED) {
      if (sp >= CG_PMT_MAX_DEPTH || !in_arena(nd.hash_off, 32, arena_len)) {
        status[t] = 3;
        return;
      }
      ld_hash_be(stk[sp], arena, lr, nd.hash_off);
      sp += 1;
      used += nd.kind == CG_PMT_INCLUDED;
    } else {
      status[t] = 3;
      return;
    }
  }
  if (sp != 1) {
    status[t] = 3;
    return;
  }
  uint32_t root[8], want[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) root[k] = stk[0][k];
  ld_hash_be(want, arena, lr, f.root_off);
  // hashesToCheck.groupBy{it} == usedHashes.groupBy{it}: equal sizes and, for every used hash,
  // equal multiplicity in both lists
  bool same = used == f.n_leaves;
  for (uint32_t j = 0; same && j < f.n_nodes; ++j) {
    const cg_pmt_node nd = nodes[f.first_node + j];
    if (nd.kind != CG_PMT_INCLUDED) continue;
    uint32_t x[8];
    ld_hash_be(x, arena, lr, nd.hash_off);
    uint32_t c_used = 0, c_check = 0;
    for (uint32_t q = 0; q < f.n_nodes; ++q) {
      const cg_pmt_node nq = nodes[f.first_node + q];
      if (nq.kind != CG_PMT_INCLUDED) continue;
      uint32_t y[8];
      ld_hash_be(y, arena, lr, nq.hash_off);
      c_used += eq8(x, y);
    }
    for (uint32_t q = 0; q < f.n_leaves; ++q) {
      uint32_t y[8];
      ld_ws(y, ws_hash, f.first_leaf + q);
      c_check += eq8(x, y);
    }
    same = c_used == c_check;
  }
  status[t] = (same && eq8(root, want)) ? 0 : 1;
}

static unsigned nblk(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

size_t ftx_ws_bytes(uint64_t n_leaves) {
  const uint64_t n = n_leaves ? n_leaves : 1;
  return ((32 * n + 255) & ~(uint64_t)255) + n + 256;
}

hipError_t launch_filtered(const cg_filtered_tx* d_ftxs, uint64_t n_ftx, const cg_pmt_node* d_nodes, uint64_t n_nodes,
                           const cg_filtered_leaf* d_leaves, uint64_t n_leaves, const uint8_t* d_arena,
                           uint64_t arena_len, uint8_t* d_status, uint8_t* d_ws, hipStream_t s) {
  if (!n_ftx) return hipSuccess;
  const uint64_t n = n_leaves ? n_leaves : 1;
  uint32_t* ws_hash = (uint32_t*)d_ws;
  uint8_t* ws_bad = d_ws + ((32 * n + 255) & ~(uint64_t)255);
  if (n_leaves)
    hipLaunchKernelGGL(k_ftx_leaves, dim3(nblk(n_leaves, 256)), dim3(256), 0, s, d_leaves, n_leaves, d_arena,
                       arena_len, ws_hash, ws_bad);
  hipLaunchKernelGGL(k_ftx_verify, dim3(nblk(n_ftx, 64)), dim3(64), 0, s, d_ftxs, n_ftx, d_nodes, n_nodes, n_leaves,
                     d_arena, arena_len, (const uint32_t*)ws_hash, (const uint8_t*)ws_bad, d_status);
  return hipGetLastError();
}

}  // namespace cg
