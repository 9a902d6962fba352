// SHA-256 / SHA-512 batch hashing and Merkle transaction ids for gfx950.
//
//   k_sha256 / k_sha512   one lane per message (SecureHash.sha256, SecureHash.kt:37)
//   k_tx_map / k_tx_leaves / k_tx_roots   WireTransaction ids: nonce_i = SHA256(salt ||
//                         BE32(i)), leaf_i = SHA256(blob_i || nonce_i) (salt leaf: SHA256(blob)),
//                         one lane per leaf; zero-hash padding to 2^k and pairwise
//                         SHA256(L || R) levels, one lane per tx
//                         (MerkleTransaction.kt:16-33,93; MerkleTree.kt:27-66)
//   k_merkle_roots        one lane per leaf list (MerkleTree.getMerkleTree)
#include <hip/hip_runtime.h>

#include "engine.h"
#include "partition.h"
#include "sha2.h"

namespace cg {

__device__ __forceinline__ uint64_t r4(uint64_t x) { return (x + 3) & ~(uint64_t)3; }

__global__ void __launch_bounds__(256) k_sha256(const cg_span* __restrict__ spans, uint64_t n,
                                                const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                uint8_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const cg_span sp = spans[i];
  uint32_t h[8];
  if (sp.off > arena_len || sp.len > arena_len - sp.off) {
    for (int k = 0; k < 8; ++k) h[k] = 0;
  } else {
    sha256_arena_suffix(h, arena, r4(arena_len), sp.off, sp.len, nullptr);
  }
  uint32_t* o = (uint32_t*)(out + 32 * i);
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = __builtin_bswap32(h[k]);
}

__global__ void __launch_bounds__(256) k_sha512(const cg_span* __restrict__ spans, uint64_t n,
                                                const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                uint8_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const cg_span sp = spans[i];
  uint64_t h[8];
  if (sp.off > arena_len || sp.len > arena_len - sp.off) {
    for (int k = 0; k < 8; ++k) h[k] = 0;
  } else {
    sha512_arena(h, arena, r4(arena_len), sp.off, sp.len);
  }
  uint32_t* o = (uint32_t*)(out + 64 * i);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    o[2 * k] = __builtin_bswap32((uint32_t)(h[k] >> 32));
    o[2 * k + 1] = __builtin_bswap32((uint32_t)h[k]);
  }
}

// SHA-256 of a 64-byte message given as 16 big-endian words (one Merkle node)
__device__ __forceinline__ void sha256_node(uint32_t out[8], const uint32_t l[8], const uint32_t r[8]) {
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

__device__ __forceinline__ void ld_node(uint32_t v[8], const uint8_t* ws, uint64_t idx) {
  const uint4* p = (const uint4*)(ws + 32 * idx);
  const uint4 a = p[0], b = p[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void st_node(uint8_t* ws, uint64_t idx, const uint32_t v[8]) {
  uint4* p = (uint4*)(ws + 32 * idx);
  p[0] = make_uint4(v[0], v[1], v[2], v[3]);
  p[1] = make_uint4(v[4], v[5], v[6], v[7]);
}

// In-place Merkle reduction of n big-endian-word leaves at ws[base .. base+n); root -> root.
__device__ void merkle_inplace(uint32_t root[8], uint8_t* ws, uint64_t base, uint32_t n) {
  if (n == 1) {
    ld_node(root, ws, base);
    return;
  }
  uint32_t m = 1;
  while (m < n) m <<= 1;
  uint32_t real = n;  // entries of the current level that are stored (the rest are zeroHash)
  while (m > 1) {
    const uint32_t half = m >> 1;
    for (uint32_t j = 0; j < half; ++j) {
      uint32_t l[8], r[8], o[8];
      if (2 * j < real) ld_node(l, ws, base + 2 * j);
      else for (int k = 0; k < 8; ++k) l[k] = 0;
      if (2 * j + 1 < real) ld_node(r, ws, base + 2 * j + 1);
      else for (int k = 0; k < 8; ++k) r[k] = 0;
      sha256_node(o, l, r);
      if (half == 1) {
        for (int k = 0; k < 8; ++k) root[k] = o[k];
      } else {
        st_node(ws, base + j, o);
      }
    }
    real = half;
    m = half;
  }
}

// ---- WireTransaction ids in three stages, so the SHA-256 work is spread one lane per leaf
// instead of one lane per transaction (a lane walking ~11 components of 80-600 bytes left
// most of each wave waiting on its longest transaction):
//   k_tx_map     one lane per tx: validity (status 1: no leaves / range outside the tables
//                / salt outside the arena); tx index of each of its components; a component
//                claimed by two transactions marks both (status 3)
//   k_tx_leaves  one lane per component: nonce = SHA256(salt || BE32(i)), leaf =
//                SHA256(blob || nonce) (salt leaf: SHA256(blob)); a blob outside the arena
//                marks its transaction (status 2)
//   k_tx_roots   one lane per tx: zero-padded pairwise levels in place -> id
// Workspace (tx_ws_bytes): leaves 32 x n_comps, the component -> tx map, the leaf order.
#define TX_NONE 0xffffffffu

__global__ void __launch_bounds__(256) k_tx_map(const cg_tx* __restrict__ txs, uint64_t n_tx, uint64_t n_comps,
                                                uint64_t arena_len, uint32_t* __restrict__ map,
                                                uint8_t* __restrict__ status) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tx) return;
  const cg_tx tx = txs[t];
  if (tx.n == 0 || tx.first > n_comps || tx.n > n_comps - tx.first || tx.salt_off > arena_len ||
      arena_len - tx.salt_off < 32) {
    status[t] = 1;
    return;
  }
  for (uint32_t i = 0; i < tx.n; ++i) {
    const uint32_t prev = atomicExch(&map[tx.first + i], (uint32_t)t);
    if (prev != TX_NONE) {
      status[t] = 3;
      status[prev] = 3;
    }
  }
}

// Leaves are hashed in order of their SHA-256 block count (class = blocks - 1, capped), so the
// 64 lanes of a wave run the same number of compressions.
#define TX_LEAF_CLASSES 16
__device__ __forceinline__ int tx_leaf_class(const uint32_t* map, const cg_component* comps, uint64_t ci) {
  if (map[ci] == TX_NONE) return -1;
  const cg_component c = comps[ci];
  const uint64_t n = (uint64_t)c.len + ((c.flags & 1u) ? 0 : 32);
  const uint64_t blocks = (n + 9 + 63) >> 6;
  return (int)(blocks > TX_LEAF_CLASSES ? TX_LEAF_CLASSES - 1 : blocks - 1);
}

__global__ void __launch_bounds__(PART_B) k_tx_leaf_count(const cg_component* __restrict__ comps, uint64_t n_comps,
                                                          const uint32_t* __restrict__ map,
                                                          uint32_t* __restrict__ bcnt) {
  const uint64_t ci = (uint64_t)blockIdx.x * PART_B + threadIdx.x;
  part_count<TX_LEAF_CLASSES>(ci < n_comps ? tx_leaf_class(map, comps, ci) : -1, bcnt);
}

__global__ void __launch_bounds__(PART_B) k_tx_leaf_scatter(const cg_component* __restrict__ comps, uint64_t n_comps,
                                                            const uint32_t* __restrict__ map,
                                                            const uint32_t* __restrict__ boff,
                                                            uint32_t* __restrict__ perm) {
  const uint64_t ci = (uint64_t)blockIdx.x * PART_B + threadIdx.x;
  part_scatter<TX_LEAF_CLASSES>(ci < n_comps ? tx_leaf_class(map, comps, ci) : -1, (uint32_t)ci, boff, perm);
}

// Message word j (big-endian) of block `blk` of blob || suffix || padding, the blob's bytes of this
// block given as 17 aligned dwords W (W[0] at the blob's 4-aligned base + 64 blk) realigned by sh8.
__device__ __forceinline__ uint32_t tx_block_word(const uint32_t* W, int j, uint32_t sh8, uint64_t blk, uint64_t len,
                                                  uint64_t n, const uint32_t* suffix_be) {
  const uint64_t pos = blk * 64 + (uint64_t)j * 4;
  const uint32_t raw = __builtin_amdgcn_alignbit(W[j + 1], W[j], sh8);  // blob bytes pos .. pos + 3
  if (pos + 4 <= len) return __builtin_bswap32(raw);
  if (suffix_be && (len & 3) == 0 && pos >= len && pos + 4 <= n) return suffix_be[(pos - len) >> 2];
  if (pos > n) return 0u;
  uint32_t acc = 0;
  for (int bb = 0; bb < 4; ++bb) {
    const uint64_t q = pos + (uint64_t)bb;
    uint32_t byte;
    if (q < len) {
      byte = (raw >> (8 * bb)) & 0xffu;
    } else if (q < n) {
      const uint64_t r = q - len;
      byte = (suffix_be[r >> 2] >> (24 - 8 * (r & 3))) & 0xffu;
    } else {
      byte = q == n ? 0x80u : 0u;
    }
    acc = (acc << 8) | byte;
  }
  return acc;
}

// One lane per component (perm order: a wave's 64 components have the same block count), the
// blob's bytes staged wave-cooperatively through LDS: for each 64-byte block, 17 consecutive lanes
// load one component's 68 aligned bytes (coalesced runs instead of 64 scattered 16-byte loads per
// instruction: round 2 moved ~4x the component bytes, profiles/r02/tx_v4), then every lane reads
// its own 17 dwords back (stride 17: no bank conflicts).
#define TX_LDS_DW 17
#ifndef TX_LEAVES_RING
#define TX_LEAVES_RING 1
#endif
__global__ void __launch_bounds__(256) k_tx_leaves(const cg_tx* __restrict__ txs, const cg_component* __restrict__ comps,
                                                   const uint32_t* __restrict__ perm,
                                                   const uint32_t* __restrict__ ranges,
                                                   const uint32_t* __restrict__ map,
                                                   const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                   uint8_t* __restrict__ status, uint8_t* __restrict__ ws) {
#if TX_LEAVES_RING
  __shared__ uint32_t ring_lds[4][2 * 64 * TX_LDS_DW];
#else
  __shared__ uint32_t stage[4][64 * TX_LDS_DW];
#endif
  __shared__ uint64_t sbase[4][64];
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t total = ranges[TX_LEAF_CLASSES];
  if ((p & ~(uint64_t)63) >= total) return;  // the whole wave is past the end
  const bool live = p < total;
  const uint64_t lr = r4(arena_len);
  uint32_t ci = 0, t = 0;
  cg_component c = {0, 0, 0};
  cg_tx tx = {0, 0, 0, 0};
  bool inside = false;
  if (live) {
    ci = perm[p];
    t = map[ci];
    tx = txs[t];
    c = comps[ci];
    inside = !(c.off > arena_len || c.len > arena_len - c.off);
    if (!inside) status[t] = 2;
  }
  const bool salt = (c.flags & 1u) != 0;
  uint32_t nonce[8];
  if (live && inside && !salt) {  // nonce = SHA256(salt || BE32(i)) : 36 bytes, one block
    uint32_t s8[8], w[16];
    sha256_init(s8);
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = __builtin_bswap32(cg_ld_bytes4(arena, lr, tx.salt_off + 4 * k));
    w[8] = (uint32_t)(ci - tx.first);
    w[9] = 0x80000000u;
#pragma unroll
    for (int k = 10; k < 15; ++k) w[k] = 0;
    w[15] = 36 * 8;
    sha256_compress(s8, w);
#pragma unroll
    for (int k = 0; k < 8; ++k) nonce[k] = s8[k];
  }
  const uint64_t len = live && inside ? c.len : 0;
  const uint64_t n = len + (salt ? 0 : 32);
  const uint32_t nbl = live && inside ? (uint32_t)((n + 9 + 63) >> 6) : 0u;
  uint32_t mbl = nbl;  // the wave's largest block count
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t x = (uint32_t)__shfl_xor((int)mbl, o, 64);
    mbl = x > mbl ? x : mbl;
  }
#if TX_LEAVES_RING
  // Round 5: each 64-B sector of a component is loaded once. The 68-B window
  // of round 3 straddled two sectors for every block, and the next block loaded the second again:
  // 2.3x the component bytes in L1 -> L2 requests, and with every XCD's waves streaming the L2
  // missed 79% of them (2.0x in memory-side reads, profiles/r05/tx/pmc). Now a ring of two sectors
  // per component in LDS: block b reads sectors b and b + 1 (dwords o .. o + 16 from the first, o =
  // the component's dword offset in its sector); sector b + 2 is loaded into registers while block b
  // compresses and written over sector b's slot afterwards. Lane l loads quarter l & 3 of the
  // sector of component 16 k + (l >> 2) for k = 0..3: four 16-B loads a lane, one 64-B request per
  // sector.
  sbase[wid][lane] = live && inside ? (c.off & ~(uint64_t)63) : ~(uint64_t)0;
  const uint32_t o = (uint32_t)(c.off & 63) >> 2;
  const uint32_t sh8 = (uint32_t)(c.off & 3) * 8u;
  uint32_t h[8];
  sha256_init(h);
  uint32_t* ring = ring_lds[wid];  // [slot][component][17 dwords: 16 + 1 pad, conflict-free reads]
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every lane's sbase is written
  __builtin_amdgcn_wave_barrier();
  auto load_sector = [&](uint64_t sec, uint4 (&r)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t cc = 16u * k + (lane >> 2), q = lane & 3u;
      const uint64_t base = sbase[wid][cc];
      const uint64_t a = base + 64ull * sec + 16ull * q;
      if (base == ~(uint64_t)0 || a >= lr) {
        r[k] = make_uint4(0, 0, 0, 0);
      } else if (a + 16 <= lr) {
        r[k] = *(const uint4*)(arena + a);
      } else {  // the arena's last partial chunk: dword by dword
        uint32_t d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) d[i] = a + 4 * i + 4 <= lr ? *(const uint32_t*)(arena + a + 4 * i) : 0u;
        r[k] = make_uint4(d[0], d[1], d[2], d[3]);
      }
    }
  };
  auto store_sector = [&](uint32_t slot, const uint4 (&r)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t cc = 16u * k + (lane >> 2), q = lane & 3u;
      uint32_t* d = ring + slot * 64 * TX_LDS_DW + cc * TX_LDS_DW + 4 * q;
      d[0] = r[k].x;
      d[1] = r[k].y;
      d[2] = r[k].z;
      d[3] = r[k].w;
    }
  };
  {
    uint4 r0[4], r1[4];
    load_sector(0, r0);
    load_sector(1, r1);
    store_sector(0, r0);
    store_sector(1, r1);
  }
  for (uint32_t blk = 0; blk < mbl; ++blk) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this block's two sectors are in LDS
    __builtin_amdgcn_wave_barrier();
    uint32_t W[TX_LDS_DW];
#pragma unroll
    for (int d = 0; d < TX_LDS_DW; ++d) {
      const uint32_t x = o + (uint32_t)d;  // dword of the two-sector window
      W[d] = ring[((blk + (x >> 4)) & 1u) * 64 * TX_LDS_DW + lane * TX_LDS_DW + (x & 15u)];
    }
    uint4 nx[4];
    const bool more = blk + 1 < mbl;  // sector blk + 2 feeds block blk + 1
    if (more) load_sector(blk + 2, nx);
    if (blk < nbl) {
      uint32_t w[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) w[j] = tx_block_word(W, j, sh8, blk, len, n, salt ? nullptr : nonce);
      if (blk + 1 == nbl) {
        w[14] = (uint32_t)((n * 8) >> 32);
        w[15] = (uint32_t)(n * 8);
      }
      sha256_compress(h, w);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every lane's window reads are done
    __builtin_amdgcn_wave_barrier();
    if (more) store_sector(blk & 1u, nx);  // sector blk + 2 over sector blk
  }
#else
  sbase[wid][lane] = live && inside ? (c.off & ~(uint64_t)3) : ~(uint64_t)0;
  const uint32_t sh8 = (uint32_t)(c.off & 3) * 8u;
  uint32_t h[8];
  sha256_init(h);
  uint32_t* st = stage[wid];
  for (uint32_t blk = 0; blk < mbl; ++blk) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous block's reads (and sbase) are done
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < TX_LDS_DW; ++k) {
      const uint32_t task = lane + 64u * k, cc = task / TX_LDS_DW, d = task % TX_LDS_DW;
      const uint64_t base = sbase[wid][cc];
      const uint64_t addr = base + 64ull * blk + 4ull * d;
      st[task] = base != ~(uint64_t)0 && addr + 4 <= lr ? *(const uint32_t*)(arena + addr) : 0u;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (blk < nbl) {
      uint32_t W[TX_LDS_DW], w[16];
#pragma unroll
      for (int d = 0; d < TX_LDS_DW; ++d) W[d] = st[lane * TX_LDS_DW + d];
#pragma unroll
      for (int j = 0; j < 16; ++j) w[j] = tx_block_word(W, j, sh8, blk, len, n, salt ? nullptr : nonce);
      if (blk + 1 == nbl) {
        w[14] = (uint32_t)((n * 8) >> 32);
        w[15] = (uint32_t)(n * 8);
      }
      sha256_compress(h, w);
    }
  }
#endif
  if (!live) return;
  if (!inside) {
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = 0;
  }
  st_node(ws, ci, h);
}

__global__ void __launch_bounds__(256) k_tx_roots(const cg_tx* __restrict__ txs, uint64_t n_tx,
                                                  uint8_t* __restrict__ ids, const uint8_t* __restrict__ status,
                                                  uint8_t* __restrict__ ws) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tx) return;
  uint32_t root[8];
  if (status[t] != 0) {
    for (int k = 0; k < 8; ++k) root[k] = 0;
  } else {
    const cg_tx tx = txs[t];
    merkle_inplace(root, ws, tx.first, tx.n);
  }
  uint32_t* o = (uint32_t*)(ids + 32 * t);
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = __builtin_bswap32(root[k]);
}

// leaves: raw digest bytes; ws holds a copy of each list (big-endian words) at first[j]
__global__ void __launch_bounds__(256) k_merkle_roots(const uint8_t* __restrict__ leaves,
                                                      const uint64_t* __restrict__ first,
                                                      const uint32_t* __restrict__ count, uint64_t n,
                                                      uint8_t* __restrict__ roots, uint8_t* __restrict__ status,
                                                      uint8_t* __restrict__ ws, const uint64_t* __restrict__ wsoff) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t cnt = count[j];
  uint32_t root[8];
  if (cnt == 0) {
    for (int k = 0; k < 8; ++k) root[k] = 0;
    status[j] = 1;
  } else {
    const uint64_t f = first[j], b = wsoff[j];
    for (uint32_t i = 0; i < cnt; ++i) {
      uint32_t v[8];
      ld_node(v, leaves, f + i);
      for (int k = 0; k < 8; ++k) v[k] = __builtin_bswap32(v[k]);
      st_node(ws, b + i, v);
    }
    merkle_inplace(root, ws, b, cnt);
    status[j] = 0;
  }
  uint32_t* o = (uint32_t*)(roots + 32 * j);
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = __builtin_bswap32(root[k]);
}

static unsigned blocks(uint64_t n) { return (unsigned)((n + 255) / 256); }

hipError_t launch_sha256(const cg_span* d_spans, uint64_t n, const uint8_t* d_arena, uint64_t arena_len,
                         uint8_t* d_out, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_sha256, dim3(blocks(n)), dim3(256), 0, s, d_spans, n, d_arena, arena_len, d_out);
  return hipGetLastError();
}

hipError_t launch_sha512(const cg_span* d_spans, uint64_t n, const uint8_t* d_arena, uint64_t arena_len,
                         uint8_t* d_out, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_sha512, dim3(blocks(n)), dim3(256), 0, s, d_spans, n, d_arena, arena_len, d_out);
  return hipGetLastError();
}

// workspace: [leaves 32 x n][map 4 x n][perm 4 x n][block class counts][ranges]
static uint64_t al256(uint64_t x) { return (x + 255) & ~(uint64_t)255; }
size_t tx_ws_bytes(uint64_t n_comps) {
  const uint64_t n = n_comps ? n_comps : 1;
  return al256(32 * n) + al256(4 * n) + al256(4 * n) + al256(4 * part_bcnt_words(TX_LEAF_CLASSES, n)) + 256;
}

hipError_t launch_tx_ids(const cg_tx* d_txs, uint64_t n_tx, const cg_component* d_comps, uint64_t n_comps,
                         const uint8_t* d_arena, uint64_t arena_len, uint8_t* d_ids, uint8_t* d_status,
                         uint8_t* d_ws, hipStream_t s) {
  if (!n_tx) return hipSuccess;
  const uint64_t n = n_comps ? n_comps : 1;
  uint32_t* map = (uint32_t*)(d_ws + al256(32 * n));
  uint32_t* perm = map + al256(4 * n) / 4;
  uint32_t* bcnt = perm + al256(4 * n) / 4;
  uint32_t* ranges = bcnt + al256(4 * part_bcnt_words(TX_LEAF_CLASSES, n)) / 4;
  hipError_t e = hipMemsetAsync(d_status, 0, n_tx, s);
  if (e == hipSuccess && n_comps) e = hipMemsetAsync(map, 0xff, 4 * n_comps, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_tx_map, dim3(blocks(n_tx)), dim3(256), 0, s, d_txs, n_tx, n_comps, arena_len, map, d_status);
  if (n_comps) {
    const uint32_t nblk = (uint32_t)((n_comps + PART_B - 1) / PART_B);
    hipLaunchKernelGGL(k_tx_leaf_count, dim3(nblk), dim3(PART_B), 0, s, d_comps, n_comps, (const uint32_t*)map, bcnt);
    hipLaunchKernelGGL(k_part_scan<TX_LEAF_CLASSES>, dim3(1), dim3(1024), 0, s, bcnt, nblk, ranges);
    hipLaunchKernelGGL(k_tx_leaf_scatter, dim3(nblk), dim3(PART_B), 0, s, d_comps, n_comps, (const uint32_t*)map,
                       (const uint32_t*)bcnt, perm);
    hipLaunchKernelGGL(k_tx_leaves, dim3(blocks(n_comps)), dim3(256), 0, s, d_txs, d_comps, (const uint32_t*)perm,
                       (const uint32_t*)ranges, (const uint32_t*)map, d_arena, arena_len, d_status, d_ws);
  }
  hipLaunchKernelGGL(k_tx_roots, dim3(blocks(n_tx)), dim3(256), 0, s, d_txs, n_tx, d_ids, (const uint8_t*)d_status,
                     d_ws);
  return hipGetLastError();
}

hipError_t launch_merkle_roots(const uint8_t* d_leaves, const uint64_t* d_first, const uint32_t* d_count, uint64_t n,
                               uint8_t* d_roots, uint8_t* d_status, uint8_t* d_ws, const uint64_t* d_wsoff,
                               hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_merkle_roots, dim3(blocks(n)), dim3(256), 0, s, d_leaves, d_first, d_count, n, d_roots,
                     d_status, d_ws, d_wsoff);
  return hipGetLastError();
}

}  // namespace cg
