// Stable device-side partition of n elements into K small classes (class -1 = dropped), in
// three passes and without per-element atomics (a hot class would serialise them):
//   part_count<K>    per block: class counts from wave ballots      -> bcnt[K][n_blocks]
//   k_part_scan      one block: exclusive scan over (class, block)  -> offsets, ranges[K + 1]
//   part_scatter<K>  per block: each element's position, input order kept within a class
// Used for the verify plan (elements = items, classes = signature schemes) and the tx-id leaf
// pass (elements = components, classes = SHA-256 block counts, so a wave hashes equal-length
// messages and no lane idles on a longer neighbour).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PART_B 256

// K class counts of this block (tot) and, per lane, how many lanes of its class precede it in
// the block (below).
template <int K>
__device__ __forceinline__ void part_block_counts(int c, uint32_t tot[K], uint32_t below[K]) {
  __shared__ uint32_t wc[PART_B / 64][K];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint64_t m = __ballot(c == k);
    if (lane == 0) wc[wave][k] = (uint32_t)__popcll(m);
    below[k] = (uint32_t)__popcll(m & lt);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    uint32_t t = 0, before = 0;
    for (uint32_t w = 0; w < PART_B / 64; ++w) {
      if (w < wave) before += wc[w][k];
      t += wc[w][k];
    }
    tot[k] = t;
    below[k] += before;
  }
}

// pass 1, body of a PART_B-thread block whose lane holds class c
template <int K>
__device__ __forceinline__ void part_count(int c, uint32_t* __restrict__ bcnt) {
  uint32_t tot[K], below[K];
  part_block_counts<K>(c, tot, below);
  if (threadIdx.x < K) bcnt[(uint64_t)threadIdx.x * gridDim.x + blockIdx.x] = tot[threadIdx.x];
}

// pass 2: one 1024-thread block; bcnt (K x n_blocks, class-major) becomes exclusive offsets;
// ranges[k] = first position of class k, ranges[K] = total
template <int K>
__global__ void __launch_bounds__(1024) k_part_scan(uint32_t* __restrict__ bcnt, uint32_t n_blocks,
                                                    uint32_t* __restrict__ ranges) {
  __shared__ uint32_t part[1024];
  const uint32_t nb = K * n_blocks;
  const uint32_t t = threadIdx.x, per = (nb + 1023) / 1024;
  const uint32_t lo = t * per < nb ? t * per : nb, hi = lo + per < nb ? lo + per : nb;
  uint32_t s = 0;
  for (uint32_t b = lo; b < hi; ++b) s += bcnt[b];
  part[t] = s;
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {
    const uint32_t v = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - s;
  for (uint32_t b = lo; b < hi; ++b) {
    if (b % n_blocks == 0) ranges[b / n_blocks] = run;
    const uint32_t v = bcnt[b];
    bcnt[b] = run;
    run += v;
  }
  if (t == 1023) ranges[K] = part[1023];
}

// pass 3, body of the same block as pass 1: element `idx` of class c -> perm
template <int K>
__device__ __forceinline__ void part_scatter(int c, uint32_t idx, const uint32_t* __restrict__ boff,
                                             uint32_t* __restrict__ perm) {
  uint32_t tot[K], below[K];
  part_block_counts<K>(c, tot, below);
  if (c >= 0) perm[boff[(uint64_t)c * gridDim.x + blockIdx.x] + below[c]] = idx;
}

static inline size_t part_bcnt_words(int k, uint64_t n) { return (size_t)k * ((n + PART_B - 1) / PART_B); }
