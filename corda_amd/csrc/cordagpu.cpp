// C ABI of the MI355X batch signature-verification engine (include/cordagpu.h).
//
// Thin host layer: argument checks, per-context device workspace, H2D/D2H for the
// host-buffer entry points, and kernel launches through engine.h. No CPU fallback: every
// verdict is computed by the HIP kernels; if the device is unusable the call fails with
// CG_ERR_DEVICE and the status bytes stay CG_NOT_RUN.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/cordagpu.h"
#include "engine.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, const char* detail = "") {
  char buf[512];
  snprintf(buf, sizeof buf, fmt, detail);
  g_err = buf;
  return code;
}

int hip_fail(hipError_t e, const char* where) {
  char buf[512];
  snprintf(buf, sizeof buf, "%s: %s", where, hipGetErrorString(e));
  g_err = buf;
  return CG_ERR_DEVICE;
}

#define HIP_TRY(expr, where)               \
  do {                                     \
    hipError_t _e = (expr);                \
    if (_e != hipSuccess) return hip_fail(_e, where); \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes + bytes / 4 + 256;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

}  // namespace

// cg_verify_batch splits a large host batch into this many consecutive item chunks: the arena
// bytes chunk k needs go H2D on a copy stream while chunk k-1 verifies.
#define CG_H2D_CHUNKS 4
#define CG_H2D_MIN_ITEMS (1u << 17)

struct cg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  cg::Fork fork = {{nullptr, nullptr, nullptr}, nullptr, {nullptr, nullptr}, {nullptr, nullptr, nullptr}, nullptr,
                   {nullptr, nullptr, nullptr}};
  std::mutex mu;
  DevBuf keyprep, itemws, btab, keys, items, arena, status, aux0, aux1, aux2;
  // transaction pipeline: verify items, spliced messages, templates; host-entry staging
  DevBuf txitems, msgs, tmpls, h_txs, h_comps, h_sigs, h_ids, h_txst;
  // tear-offs: leaf-hash workspace
  DevBuf ftxws;
  // host-buffer verify: a copy stream and one event per arena segment (chunked H2D / verify)
  hipStream_t copy = nullptr;
  hipEvent_t seg[CG_H2D_CHUNKS + 1] = {};
};

extern "C" {

int cg_abi_version(void) { return CG_ABI_VERSION; }

const char* cg_build_info(void) {
  return "corda_amd libcordagpu: HIP kernels for gfx950 (Ed25519 i2p-0.2.0 semantics, ECDSA BC-1.57 semantics, "
         "SHA-256/512, Merkle tx ids)";
}

int cg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* cg_last_error(void) { return g_err.c_str(); }

int cg_open(cg_ctx** out, const cg_config* cfg) {
  if (!out) return fail(CG_ERR_ARG, "cg_open: out is NULL");
  *out = nullptr;
  int dev = cfg ? cfg->device : 0;
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n), "hipGetDeviceCount");
  if (dev < 0 || dev >= n) return fail(CG_ERR_ARG, "cg_open: device ordinal out of range");
  HIP_TRY(hipSetDevice(dev), "hipSetDevice");
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, dev), "hipGetDeviceProperties");
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(CG_ERR_DEVICE, "cg_open: kernels are built for gfx950, device is %s", prop.gcnArchName);
  cg_ctx* c = new cg_ctx();
  c->device = dev;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return hip_fail(e, "hipStreamCreate");
  }
  for (int k = 0; k < 3 && e == hipSuccess; ++k) e = hipStreamCreateWithFlags(&c->fork.side[k], hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork.start, hipEventDisableTiming);
  for (int k = 0; k < 2 && e == hipSuccess; ++k)
    e = hipEventCreateWithFlags(&c->fork.ec_decoded[k], hipEventDisableTiming);
  for (int k = 0; k < 3 && e == hipSuccess; ++k) e = hipEventCreateWithFlags(&c->fork.ready[k], hipEventDisableTiming);
  for (int k = 0; k < 3 && e == hipSuccess; ++k) e = hipEventCreateWithFlags(&c->fork.row0[k], hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork.front, hipEventDisableTiming);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking);
  for (int k = 0; k <= CG_H2D_CHUNKS && e == hipSuccess; ++k)
    e = hipEventCreateWithFlags(&c->seg[k], hipEventDisableTiming);
  if (e == hipSuccess) e = cg::upload_constants();
  if (e == hipSuccess) e = c->btab.ensure(cg::btab_bytes());
  if (e == hipSuccess) e = cg::init_btab(c->btab.p, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    const int rc = hip_fail(e, "side streams / upload_constants / base-point tables");
    cg_close(c);
    return rc;
  }
  *out = c;
  return CG_OK;
}

void cg_close(cg_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  c->keyprep.release();
  c->itemws.release();
  c->btab.release();
  c->keys.release();
  c->items.release();
  c->arena.release();
  c->status.release();
  c->aux0.release();
  c->aux1.release();
  c->aux2.release();
  for (DevBuf* b : {&c->txitems, &c->msgs, &c->tmpls, &c->h_txs, &c->h_comps, &c->h_sigs, &c->h_ids, &c->h_txst, &c->ftxws})
    b->release();
  for (int k = 0; k < 3; ++k) {
    if (c->fork.side[k]) {
      hipStreamSynchronize(c->fork.side[k]);
      hipStreamDestroy(c->fork.side[k]);
    }
    if (c->fork.ready[k]) hipEventDestroy(c->fork.ready[k]);
    if (c->fork.row0[k]) hipEventDestroy(c->fork.row0[k]);
  }
  if (c->fork.start) hipEventDestroy(c->fork.start);
  if (c->fork.front) hipEventDestroy(c->fork.front);
  if (c->copy) {
    hipStreamSynchronize(c->copy);
    hipStreamDestroy(c->copy);
  }
  for (int k = 0; k <= CG_H2D_CHUNKS; ++k)
    if (c->seg[k]) hipEventDestroy(c->seg[k]);
  for (int k = 0; k < 2; ++k)
    if (c->fork.ec_decoded[k]) hipEventDestroy(c->fork.ec_decoded[k]);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
}

int cg_reserve(cg_ctx* c, uint32_t max_keys, uint64_t max_items) {
  if (!c) return fail(CG_ERR_ARG, "cg_reserve: ctx is NULL");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  HIP_TRY(c->keyprep.ensure(cg::keyprep_bytes(max_keys)), "hipMalloc(keyprep)");
  HIP_TRY(c->itemws.ensure(cg::item_ws_bytes(max_items)), "hipMalloc(item workspace)");
  return CG_OK;
}

int cg_verify_batch_device(cg_ctx* c, const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items,
                           uint64_t n_items, const uint8_t* d_arena, uint64_t arena_len, uint32_t mode,
                           uint8_t* d_status, void* hip_stream) {
  if (!c) return fail(CG_ERR_ARG, "cg_verify_batch_device: ctx is NULL");
  if (n_items && (!d_items || !d_status)) return fail(CG_ERR_ARG, "cg_verify_batch_device: NULL buffer");
  if (mode > CG_MODE_ISVALID) return fail(CG_ERR_ARG, "cg_verify_batch_device: bad mode");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  if (c->keyprep.cap < cg::keyprep_bytes(n_keys) || c->itemws.cap < cg::item_ws_bytes(n_items)) {
    // growing the workspace synchronises the device; cg_reserve ahead of time avoids it
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    HIP_TRY(c->keyprep.ensure(cg::keyprep_bytes(n_keys)), "hipMalloc(keyprep)");
    HIP_TRY(c->itemws.ensure(cg::item_ws_bytes(n_items)), "hipMalloc(item workspace)");
  }
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
  HIP_TRY(cg::launch_verify(d_keys, n_keys, d_items, n_items, d_arena, arena_len, mode, d_status, c->keyprep.p,
                            c->itemws.p, c->btab.p, s, nullptr, 0, &c->fork),
          "launch_verify");
  return CG_OK;
}

int cg_prepare_keys_device(cg_ctx* c, const cg_key* d_keys, uint32_t n_keys, const uint8_t* d_arena,
                           uint64_t arena_len, void* hip_stream) {
  if (!c) return fail(CG_ERR_ARG, "cg_prepare_keys_device: ctx is NULL");
  if (n_keys && !d_keys) return fail(CG_ERR_ARG, "cg_prepare_keys_device: keys is NULL");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  if (c->keyprep.cap < cg::keyprep_bytes(n_keys)) {
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    HIP_TRY(c->keyprep.ensure(cg::keyprep_bytes(n_keys)), "hipMalloc(keyprep)");
  }
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
  HIP_TRY(cg::launch_keyprep(d_keys, n_keys, d_arena, arena_len, c->keyprep.p, s, &c->fork), "launch_keyprep");
  return CG_OK;
}

int cg_verify_items_device(cg_ctx* c, const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items,
                           uint64_t n_items, const uint8_t* d_arena, uint64_t arena_len, uint32_t mode,
                           uint8_t* d_status, void* hip_stream) {
  if (!c) return fail(CG_ERR_ARG, "cg_verify_items_device: ctx is NULL");
  if (n_items && (!d_items || !d_status)) return fail(CG_ERR_ARG, "cg_verify_items_device: NULL buffer");
  if (mode > CG_MODE_ISVALID) return fail(CG_ERR_ARG, "cg_verify_items_device: bad mode");
  std::lock_guard<std::mutex> g(c->mu);
  if (c->keyprep.cap < cg::keyprep_bytes(n_keys))
    return fail(CG_ERR_ARG, "cg_verify_items_device: keys were not prepared (call cg_prepare_keys_device)");
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  if (c->itemws.cap < cg::item_ws_bytes(n_items)) {
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    HIP_TRY(c->itemws.ensure(cg::item_ws_bytes(n_items)), "hipMalloc(item workspace)");
  }
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
  HIP_TRY(cg::launch_items(d_keys, n_keys, d_items, n_items, d_arena, arena_len, mode, d_status, c->keyprep.p,
                           c->itemws.p, c->btab.p, s, nullptr, 0, &c->fork),
          "launch_items");
  return CG_OK;
}

int cg_verify_batch(cg_ctx* c, const cg_key* keys, uint32_t n_keys, const cg_item* items, uint64_t n_items,
                    const uint8_t* arena, uint64_t arena_len, uint32_t mode, uint8_t* status_out,
                    cg_stats* stats) {
  if (!c) return fail(CG_ERR_ARG, "cg_verify_batch: ctx is NULL");
  if (n_items && (!items || !status_out)) return fail(CG_ERR_ARG, "cg_verify_batch: NULL buffer");
  if (n_keys && !keys) return fail(CG_ERR_ARG, "cg_verify_batch: keys is NULL");
  if (arena_len && !arena) return fail(CG_ERR_ARG, "cg_verify_batch: arena is NULL");
  if (mode > CG_MODE_ISVALID) return fail(CG_ERR_ARG, "cg_verify_batch: bad mode");
  for (uint64_t i = 0; i < n_items; ++i) status_out[i] = CG_NOT_RUN;
  if (n_items == 0) return CG_OK;
  auto t0 = std::chrono::steady_clock::now();
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  const size_t arena_alloc = ((arena_len + 3) & ~(uint64_t)3) + 16;
  HIP_TRY(c->keys.ensure(sizeof(cg_key) * (n_keys ? n_keys : 1)), "hipMalloc(keys)");
  HIP_TRY(c->items.ensure(sizeof(cg_item) * n_items), "hipMalloc(items)");
  HIP_TRY(c->arena.ensure(arena_alloc), "hipMalloc(arena)");
  HIP_TRY(c->status.ensure(n_items), "hipMalloc(status)");
  HIP_TRY(c->keyprep.ensure(cg::keyprep_bytes(n_keys)), "hipMalloc(keyprep)");
  HIP_TRY(c->itemws.ensure(cg::item_ws_bytes(n_items)), "hipMalloc(item workspace)");
  hipStream_t s = c->stream;
  hipEvent_t ev[4];
  for (auto& e : ev) HIP_TRY(hipEventCreate(&e), "hipEventCreate");
  // Chunk plan: item chunk k needs arena[0 .. need[k]) (prefix max of its items' extents,
  // clamped to the arena: an item outside it is CG_NOT_RUN and reads nothing); key prep needs
  // arena[0 .. key_end). Pipelined only when the keys sit in the first quarter of the arena,
  // which is how a caller appending (key, sig, clear) in order lays it out; otherwise one copy.
  uint64_t key_end = 0;
  for (uint32_t k = 0; k < n_keys; ++k) {
    const uint64_t e = keys[k].off > arena_len ? arena_len : keys[k].off + keys[k].len;
    key_end = e > key_end ? e : key_end;
  }
  key_end = key_end < arena_len ? key_end : arena_len;
  int chunks = (n_items >= CG_H2D_MIN_ITEMS && key_end <= arena_len / 4) ? CG_H2D_CHUNKS : 1;
  uint64_t first[CG_H2D_CHUNKS + 1], need[CG_H2D_CHUNKS];
  for (int k = 0; k <= chunks; ++k) first[k] = n_items * (uint64_t)k / (uint64_t)chunks;
  uint64_t run = key_end;
  for (int k = 0; k < chunks; ++k) {
    for (uint64_t i = first[k]; i < first[k + 1]; ++i) {
      const cg_item& it = items[i];
      const uint64_t se = it.sig_off > arena_len ? 0 : it.sig_off + it.sig_len;
      const uint64_t me = it.msg_off > arena_len ? 0 : it.msg_off + it.msg_len;
      const uint64_t e = se > me ? se : me;
      if (e > run) run = e;
    }
    need[k] = run < arena_len ? run : arena_len;
  }
  if (chunks == 1) need[0] = arena_len;
  HIP_TRY(hipEventRecord(ev[0], s), "hipEventRecord");
  HIP_TRY(hipStreamWaitEvent(c->copy, ev[0], 0), "hipStreamWaitEvent");
  if (n_keys)
    HIP_TRY(hipMemcpyAsync(c->keys.p, keys, sizeof(cg_key) * n_keys, hipMemcpyHostToDevice, c->copy), "H2D keys");
  HIP_TRY(hipMemcpyAsync(c->items.p, items, sizeof(cg_item) * n_items, hipMemcpyHostToDevice, c->copy), "H2D items");
  uint64_t copied = 0;
  for (int k = 0; k < chunks; ++k) {
    if (need[k] > copied) {
      HIP_TRY(hipMemcpyAsync((uint8_t*)c->arena.p + copied, arena + copied, need[k] - copied, hipMemcpyHostToDevice,
                             c->copy), "H2D arena");
      copied = need[k];
    }
    HIP_TRY(hipEventRecord(c->seg[k], c->copy), "hipEventRecord");
    HIP_TRY(hipStreamWaitEvent(s, c->seg[k], 0), "hipStreamWaitEvent");
    if (k == 0) {
      HIP_TRY(hipEventRecord(ev[1], s), "hipEventRecord");
      // key tables sized by every item's key (not just chunk 0's)
      HIP_TRY(cg::launch_keyprep((const cg_key*)c->keys.p, n_keys, (const uint8_t*)c->arena.p, arena_len, c->keyprep.p,
                                 s, &c->fork, (const cg_item*)c->items.p, n_items), "launch_keyprep");
    }
    HIP_TRY(cg::launch_items((const cg_key*)c->keys.p, n_keys, (const cg_item*)c->items.p + first[k],
                             first[k + 1] - first[k], (const uint8_t*)c->arena.p, arena_len, mode,
                             (uint8_t*)c->status.p + first[k], c->keyprep.p, c->itemws.p, c->btab.p, s, nullptr, 0,
                             &c->fork), "launch_items");
  }
  HIP_TRY(hipEventRecord(ev[2], s), "hipEventRecord");
  HIP_TRY(hipMemcpyAsync(status_out, c->status.p, n_items, hipMemcpyDeviceToHost, s), "D2H status");
  HIP_TRY(hipEventRecord(ev[3], s), "hipEventRecord");
  HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
  if (stats) {
    float a = 0, b = 0, d = 0;
    hipEventElapsedTime(&a, ev[0], ev[1]);
    hipEventElapsedTime(&b, ev[1], ev[2]);
    hipEventElapsedTime(&d, ev[2], ev[3]);
    stats->n_items = n_items;
    stats->n_keys = n_keys;
    stats->ms_h2d = a;
    stats->ms_key_prep = 0;
    stats->ms_verify = b;
    stats->ms_d2h = d;
    stats->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  for (auto& e : ev) hipEventDestroy(e);
  return CG_OK;
}

int cg_sha256_batch_device(cg_ctx* c, const cg_span* d_spans, uint64_t n, const uint8_t* d_arena,
                           uint64_t arena_len, uint8_t* d_digests, void* hip_stream) {
  if (!c) return fail(CG_ERR_ARG, "cg_sha256_batch_device: ctx is NULL");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
  HIP_TRY(cg::launch_sha256(d_spans, n, d_arena, arena_len, d_digests, s), "launch_sha256");
  return CG_OK;
}

static int hash_batch(cg_ctx* c, const cg_span* spans, uint64_t n, const uint8_t* arena, uint64_t arena_len,
                      uint8_t* out, int which) {
  if (!c) return fail(CG_ERR_ARG, "hash batch: ctx is NULL");
  if (n && (!spans || !out)) return fail(CG_ERR_ARG, "hash batch: NULL buffer");
  if (n == 0) return CG_OK;
  const size_t dlen = which == 256 ? 32 : 64;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  HIP_TRY(c->items.ensure(sizeof(cg_span) * n), "hipMalloc(spans)");
  HIP_TRY(c->arena.ensure(((arena_len + 3) & ~(uint64_t)3) + 16), "hipMalloc(arena)");
  HIP_TRY(c->aux0.ensure(dlen * n), "hipMalloc(digests)");
  HIP_TRY(hipMemcpyAsync(c->items.p, spans, sizeof(cg_span) * n, hipMemcpyHostToDevice, s), "H2D spans");
  if (arena_len) HIP_TRY(hipMemcpyAsync(c->arena.p, arena, arena_len, hipMemcpyHostToDevice, s), "H2D arena");
  if (which == 256)
    HIP_TRY(cg::launch_sha256((const cg_span*)c->items.p, n, (const uint8_t*)c->arena.p, arena_len,
                              (uint8_t*)c->aux0.p, s), "launch_sha256");
  else
    HIP_TRY(cg::launch_sha512((const cg_span*)c->items.p, n, (const uint8_t*)c->arena.p, arena_len,
                              (uint8_t*)c->aux0.p, s), "launch_sha512");
  HIP_TRY(hipMemcpyAsync(out, c->aux0.p, dlen * n, hipMemcpyDeviceToHost, s), "D2H digests");
  HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
  return CG_OK;
}

int cg_sha256_batch(cg_ctx* c, const cg_span* spans, uint64_t n, const uint8_t* arena, uint64_t arena_len,
                    uint8_t* out) {
  return hash_batch(c, spans, n, arena, arena_len, out, 256);
}
int cg_sha512_batch(cg_ctx* c, const cg_span* spans, uint64_t n, const uint8_t* arena, uint64_t arena_len,
                    uint8_t* out) {
  return hash_batch(c, spans, n, arena, arena_len, out, 512);
}

int cg_tx_ids_device(cg_ctx* c, const cg_tx* d_txs, uint64_t n_tx, const cg_component* d_comps, uint64_t n_comps,
                     const uint8_t* d_arena, uint64_t arena_len, uint8_t* d_ids, uint8_t* d_status,
                     void* hip_stream) {
  if (!c) return fail(CG_ERR_ARG, "cg_tx_ids_device: ctx is NULL");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  if (c->aux2.cap < cg::tx_ws_bytes(n_comps)) {
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    HIP_TRY(c->aux2.ensure(cg::tx_ws_bytes(n_comps)), "hipMalloc(leaf ws)");
  }
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
  HIP_TRY(cg::launch_tx_ids(d_txs, n_tx, d_comps, n_comps, d_arena, arena_len, d_ids, d_status,
                            (uint8_t*)c->aux2.p, s), "launch_tx_ids");
  return CG_OK;
}

int cg_tx_ids(cg_ctx* c, const cg_tx* txs, uint64_t n_tx, const cg_component* comps, uint64_t n_comps,
              const uint8_t* arena, uint64_t arena_len, uint8_t* ids_out, uint8_t* status_out) {
  if (!c) return fail(CG_ERR_ARG, "cg_tx_ids: ctx is NULL");
  if (n_tx && (!txs || !ids_out || !status_out)) return fail(CG_ERR_ARG, "cg_tx_ids: NULL buffer");
  if (n_tx == 0) return CG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  HIP_TRY(c->keys.ensure(sizeof(cg_tx) * n_tx), "hipMalloc(txs)");
  HIP_TRY(c->items.ensure(sizeof(cg_component) * (n_comps ? n_comps : 1)), "hipMalloc(comps)");
  HIP_TRY(c->arena.ensure(((arena_len + 3) & ~(uint64_t)3) + 16), "hipMalloc(arena)");
  HIP_TRY(c->aux0.ensure(32 * n_tx), "hipMalloc(ids)");
  HIP_TRY(c->status.ensure(n_tx), "hipMalloc(status)");
  HIP_TRY(c->aux2.ensure(cg::tx_ws_bytes(n_comps)), "hipMalloc(leaf ws)");
  HIP_TRY(hipMemcpyAsync(c->keys.p, txs, sizeof(cg_tx) * n_tx, hipMemcpyHostToDevice, s), "H2D txs");
  if (n_comps)
    HIP_TRY(hipMemcpyAsync(c->items.p, comps, sizeof(cg_component) * n_comps, hipMemcpyHostToDevice, s), "H2D comps");
  if (arena_len) HIP_TRY(hipMemcpyAsync(c->arena.p, arena, arena_len, hipMemcpyHostToDevice, s), "H2D arena");
  HIP_TRY(cg::launch_tx_ids((const cg_tx*)c->keys.p, n_tx, (const cg_component*)c->items.p, n_comps,
                            (const uint8_t*)c->arena.p, arena_len, (uint8_t*)c->aux0.p, (uint8_t*)c->status.p,
                            (uint8_t*)c->aux2.p, s), "launch_tx_ids");
  HIP_TRY(hipMemcpyAsync(ids_out, c->aux0.p, 32 * n_tx, hipMemcpyDeviceToHost, s), "D2H ids");
  HIP_TRY(hipMemcpyAsync(status_out, c->status.p, n_tx, hipMemcpyDeviceToHost, s), "D2H status");
  HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
  return CG_OK;
}

int cg_merkle_roots(cg_ctx* c, const uint8_t* leaves, const uint64_t* first, const uint32_t* count, uint64_t n,
                    uint8_t* roots_out, uint8_t* status_out) {
  if (!c) return fail(CG_ERR_ARG, "cg_merkle_roots: ctx is NULL");
  if (n && (!first || !count || !roots_out || !status_out)) return fail(CG_ERR_ARG, "cg_merkle_roots: NULL buffer");
  if (n == 0) return CG_OK;
  uint64_t total = 0, ws = 0;
  std::vector<uint64_t> wsoff(n);
  for (uint64_t j = 0; j < n; ++j) {
    if (first[j] + count[j] > total) total = first[j] + count[j];
    wsoff[j] = ws;
    ws += count[j];
  }
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  HIP_TRY(c->arena.ensure(32 * (total ? total : 1)), "hipMalloc(leaves)");
  HIP_TRY(c->keys.ensure(8 * n), "hipMalloc(first)");
  HIP_TRY(c->items.ensure(4 * n), "hipMalloc(count)");
  HIP_TRY(c->aux0.ensure(32 * n), "hipMalloc(roots)");
  HIP_TRY(c->status.ensure(n), "hipMalloc(status)");
  HIP_TRY(c->aux1.ensure(32 * (ws ? ws : 1)), "hipMalloc(ws)");
  HIP_TRY(c->aux2.ensure(8 * n), "hipMalloc(wsoff)");
  if (total) HIP_TRY(hipMemcpyAsync(c->arena.p, leaves, 32 * total, hipMemcpyHostToDevice, s), "H2D leaves");
  HIP_TRY(hipMemcpyAsync(c->keys.p, first, 8 * n, hipMemcpyHostToDevice, s), "H2D first");
  HIP_TRY(hipMemcpyAsync(c->items.p, count, 4 * n, hipMemcpyHostToDevice, s), "H2D count");
  HIP_TRY(hipMemcpyAsync(c->aux2.p, wsoff.data(), 8 * n, hipMemcpyHostToDevice, s), "H2D wsoff");
  HIP_TRY(cg::launch_merkle_roots((const uint8_t*)c->arena.p, (const uint64_t*)c->keys.p, (const uint32_t*)c->items.p,
                                  n, (uint8_t*)c->aux0.p, (uint8_t*)c->status.p, (uint8_t*)c->aux1.p,
                                  (const uint64_t*)c->aux2.p, s),
          "launch_merkle_roots");
  HIP_TRY(hipMemcpyAsync(roots_out, c->aux0.p, 32 * n, hipMemcpyDeviceToHost, s), "D2H roots");
  HIP_TRY(hipMemcpyAsync(status_out, c->status.p, n, hipMemcpyDeviceToHost, s), "D2H status");
  HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
  return CG_OK;
}

// cg_verify_transactions_device with the ctx lock held
static int verify_transactions_locked(cg_ctx* c, const cg_tx* d_txs, uint64_t n_tx, const cg_component* d_comps,
                                      uint64_t n_comps, const cg_key* d_keys, uint32_t n_keys, const cg_txsig* d_sigs,
                                      uint64_t n_sigs, const cg_signable_tmpl* tmpls, uint32_t n_tmpls,
                                      const uint8_t* d_arena, uint64_t arena_len, uint32_t mode, uint8_t* d_ids,
                                      uint8_t* d_tx_status, uint8_t* d_sig_status, hipStream_t s) {
  uint64_t maxlen = 0;
  for (uint32_t k = 0; k < n_tmpls; ++k) {
    const uint64_t l = (uint64_t)tmpls[k].prefix_len + 32u + tmpls[k].suffix_len;
    if (l > maxlen) maxlen = l;
  }
  uint64_t slot = (maxlen + 15) & ~(uint64_t)15;
  if (slot == 0) slot = 16;
  const size_t need_leaf = cg::tx_ws_bytes(n_comps), need_items = sizeof(cg_item) * (n_sigs ? n_sigs : 1),
               need_msgs = slot * (n_sigs ? n_sigs : 1), need_tmpl = sizeof(cg_signable_tmpl) * (n_tmpls ? n_tmpls : 1);
  if (c->aux2.cap < need_leaf || c->txitems.cap < need_items || c->msgs.cap < need_msgs ||
      c->tmpls.cap < need_tmpl || c->keyprep.cap < cg::keyprep_bytes(n_keys) ||
      c->itemws.cap < cg::item_ws_bytes(n_sigs)) {
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    HIP_TRY(c->aux2.ensure(need_leaf), "hipMalloc(leaf ws)");
    HIP_TRY(c->txitems.ensure(need_items), "hipMalloc(tx items)");
    HIP_TRY(c->msgs.ensure(need_msgs), "hipMalloc(spliced messages)");
    HIP_TRY(c->tmpls.ensure(need_tmpl), "hipMalloc(templates)");
    HIP_TRY(c->keyprep.ensure(cg::keyprep_bytes(n_keys)), "hipMalloc(keyprep)");
    HIP_TRY(c->itemws.ensure(cg::item_ws_bytes(n_sigs)), "hipMalloc(item workspace)");
  }
  if (n_tmpls)
    HIP_TRY(hipMemcpyAsync(c->tmpls.p, tmpls, sizeof(cg_signable_tmpl) * n_tmpls, hipMemcpyHostToDevice, s),
            "H2D templates");
  HIP_TRY(cg::launch_tx_ids(d_txs, n_tx, d_comps, n_comps, d_arena, arena_len, d_ids, d_tx_status,
                            (uint8_t*)c->aux2.p, s), "launch_tx_ids");
  if (n_sigs == 0) return CG_OK;
  HIP_TRY(cg::launch_tx_sig_items(d_sigs, n_sigs, (const cg_signable_tmpl*)c->tmpls.p, n_tmpls, d_tx_status, n_tx,
                                  d_ids, d_arena, arena_len, slot, (cg_item*)c->txitems.p, (uint8_t*)c->msgs.p, s),
          "launch_tx_sig_items");
  HIP_TRY(cg::launch_verify(d_keys, n_keys, (const cg_item*)c->txitems.p, n_sigs, d_arena, arena_len, mode,
                            d_sig_status, c->keyprep.p, c->itemws.p, c->btab.p, s, (const uint8_t*)c->msgs.p,
                            slot * n_sigs, &c->fork),
          "launch_verify");
  return CG_OK;
}

int cg_verify_transactions_device(cg_ctx* c, const cg_tx* d_txs, uint64_t n_tx, const cg_component* d_comps,
                                  uint64_t n_comps, const cg_key* d_keys, uint32_t n_keys, const cg_txsig* d_sigs,
                                  uint64_t n_sigs, const cg_signable_tmpl* tmpls, uint32_t n_tmpls,
                                  const uint8_t* d_arena, uint64_t arena_len, uint32_t mode, uint8_t* d_ids,
                                  uint8_t* d_tx_status, uint8_t* d_sig_status, void* hip_stream) {
  if (!c) return fail(CG_ERR_ARG, "cg_verify_transactions_device: ctx is NULL");
  if (n_tx && (!d_txs || !d_ids || !d_tx_status)) return fail(CG_ERR_ARG, "cg_verify_transactions_device: NULL tx buffer");
  if (n_sigs && (!d_sigs || !d_sig_status)) return fail(CG_ERR_ARG, "cg_verify_transactions_device: NULL sig buffer");
  if (n_tmpls && !tmpls) return fail(CG_ERR_ARG, "cg_verify_transactions_device: templates is NULL");
  if (mode > CG_MODE_ISVALID) return fail(CG_ERR_ARG, "cg_verify_transactions_device: bad mode");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
  return verify_transactions_locked(c, d_txs, n_tx, d_comps, n_comps, d_keys, n_keys, d_sigs, n_sigs, tmpls, n_tmpls,
                                    d_arena, arena_len, mode, d_ids, d_tx_status, d_sig_status, s);
}

int cg_verify_transactions(cg_ctx* c, const cg_tx* txs, uint64_t n_tx, const cg_component* comps, uint64_t n_comps,
                           const cg_key* keys, uint32_t n_keys, const cg_txsig* sigs, uint64_t n_sigs,
                           const cg_signable_tmpl* tmpls, uint32_t n_tmpls, const uint8_t* arena,
                           uint64_t arena_len, uint32_t mode, uint8_t* ids_out, uint8_t* tx_status_out,
                           uint8_t* sig_status_out) {
  if (!c) return fail(CG_ERR_ARG, "cg_verify_transactions: ctx is NULL");
  if (n_tx && (!txs || !ids_out || !tx_status_out)) return fail(CG_ERR_ARG, "cg_verify_transactions: NULL tx buffer");
  if (n_sigs && (!sigs || !sig_status_out)) return fail(CG_ERR_ARG, "cg_verify_transactions: NULL sig buffer");
  if (n_comps && !comps) return fail(CG_ERR_ARG, "cg_verify_transactions: comps is NULL");
  if (n_keys && !keys) return fail(CG_ERR_ARG, "cg_verify_transactions: keys is NULL");
  if (n_tmpls && !tmpls) return fail(CG_ERR_ARG, "cg_verify_transactions: templates is NULL");
  if (arena_len && !arena) return fail(CG_ERR_ARG, "cg_verify_transactions: arena is NULL");
  if (mode > CG_MODE_ISVALID) return fail(CG_ERR_ARG, "cg_verify_transactions: bad mode");
  for (uint64_t i = 0; i < n_sigs; ++i) sig_status_out[i] = CG_NOT_RUN;
  if (n_tx == 0 && n_sigs == 0) return CG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  HIP_TRY(c->h_txs.ensure(sizeof(cg_tx) * (n_tx ? n_tx : 1)), "hipMalloc(txs)");
  HIP_TRY(c->h_comps.ensure(sizeof(cg_component) * (n_comps ? n_comps : 1)), "hipMalloc(comps)");
  HIP_TRY(c->keys.ensure(sizeof(cg_key) * (n_keys ? n_keys : 1)), "hipMalloc(keys)");
  HIP_TRY(c->h_sigs.ensure(sizeof(cg_txsig) * (n_sigs ? n_sigs : 1)), "hipMalloc(sigs)");
  HIP_TRY(c->arena.ensure(((arena_len + 3) & ~(uint64_t)3) + 16), "hipMalloc(arena)");
  HIP_TRY(c->h_ids.ensure(32 * (n_tx ? n_tx : 1)), "hipMalloc(ids)");
  HIP_TRY(c->h_txst.ensure(n_tx ? n_tx : 1), "hipMalloc(tx status)");
  HIP_TRY(c->status.ensure(n_sigs ? n_sigs : 1), "hipMalloc(sig status)");
  if (n_tx) HIP_TRY(hipMemcpyAsync(c->h_txs.p, txs, sizeof(cg_tx) * n_tx, hipMemcpyHostToDevice, s), "H2D txs");
  if (n_comps)
    HIP_TRY(hipMemcpyAsync(c->h_comps.p, comps, sizeof(cg_component) * n_comps, hipMemcpyHostToDevice, s),
            "H2D comps");
  if (n_keys) HIP_TRY(hipMemcpyAsync(c->keys.p, keys, sizeof(cg_key) * n_keys, hipMemcpyHostToDevice, s), "H2D keys");
  if (n_sigs)
    HIP_TRY(hipMemcpyAsync(c->h_sigs.p, sigs, sizeof(cg_txsig) * n_sigs, hipMemcpyHostToDevice, s), "H2D sigs");
  if (arena_len) HIP_TRY(hipMemcpyAsync(c->arena.p, arena, arena_len, hipMemcpyHostToDevice, s), "H2D arena");
  int rc = verify_transactions_locked(c, (const cg_tx*)c->h_txs.p, n_tx, (const cg_component*)c->h_comps.p, n_comps,
                                      (const cg_key*)c->keys.p, n_keys, (const cg_txsig*)c->h_sigs.p, n_sigs, tmpls,
                                      n_tmpls, (const uint8_t*)c->arena.p, arena_len, mode, (uint8_t*)c->h_ids.p,
                                      (uint8_t*)c->h_txst.p, (uint8_t*)c->status.p, s);
  if (rc != CG_OK) return rc;
  if (n_tx) {
    HIP_TRY(hipMemcpyAsync(ids_out, c->h_ids.p, 32 * n_tx, hipMemcpyDeviceToHost, s), "D2H ids");
    HIP_TRY(hipMemcpyAsync(tx_status_out, c->h_txst.p, n_tx, hipMemcpyDeviceToHost, s), "D2H tx status");
  }
  if (n_sigs) HIP_TRY(hipMemcpyAsync(sig_status_out, c->status.p, n_sigs, hipMemcpyDeviceToHost, s), "D2H sig status");
  HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
  return CG_OK;
}

int cg_verify_filtered_device(cg_ctx* c, const cg_filtered_tx* d_ftxs, uint64_t n_ftx, const cg_pmt_node* d_nodes,
                              uint64_t n_nodes, const cg_filtered_leaf* d_leaves, uint64_t n_leaves,
                              const uint8_t* d_arena, uint64_t arena_len, uint8_t* d_status, void* hip_stream) {
  if (!c) return fail(CG_ERR_ARG, "cg_verify_filtered_device: ctx is NULL");
  if (n_ftx && (!d_ftxs || !d_status)) return fail(CG_ERR_ARG, "cg_verify_filtered_device: NULL buffer");
  if (n_ftx == 0) return CG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  if (c->ftxws.cap < cg::ftx_ws_bytes(n_leaves)) {
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    HIP_TRY(c->ftxws.ensure(cg::ftx_ws_bytes(n_leaves)), "hipMalloc(filtered ws)");
  }
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
  HIP_TRY(cg::launch_filtered(d_ftxs, n_ftx, d_nodes, n_nodes, d_leaves, n_leaves, d_arena, arena_len, d_status,
                              (uint8_t*)c->ftxws.p, s), "launch_filtered");
  return CG_OK;
}

int cg_verify_filtered(cg_ctx* c, const cg_filtered_tx* ftxs, uint64_t n_ftx, const cg_pmt_node* nodes,
                       uint64_t n_nodes, const cg_filtered_leaf* leaves, uint64_t n_leaves, const uint8_t* arena,
                       uint64_t arena_len, uint8_t* status_out) {
  if (!c) return fail(CG_ERR_ARG, "cg_verify_filtered: ctx is NULL");
  if (n_ftx && (!ftxs || !status_out)) return fail(CG_ERR_ARG, "cg_verify_filtered: NULL buffer");
  if ((n_nodes && !nodes) || (n_leaves && !leaves) || (arena_len && !arena))
    return fail(CG_ERR_ARG, "cg_verify_filtered: NULL table");
  if (n_ftx == 0) return CG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  HIP_TRY(c->h_txs.ensure(sizeof(cg_filtered_tx) * n_ftx), "hipMalloc(filtered txs)");
  HIP_TRY(c->h_comps.ensure(sizeof(cg_pmt_node) * (n_nodes ? n_nodes : 1)), "hipMalloc(nodes)");
  HIP_TRY(c->h_sigs.ensure(sizeof(cg_filtered_leaf) * (n_leaves ? n_leaves : 1)), "hipMalloc(leaves)");
  HIP_TRY(c->arena.ensure(((arena_len + 3) & ~(uint64_t)3) + 16), "hipMalloc(arena)");
  HIP_TRY(c->status.ensure(n_ftx), "hipMalloc(status)");
  HIP_TRY(c->ftxws.ensure(cg::ftx_ws_bytes(n_leaves)), "hipMalloc(filtered ws)");
  HIP_TRY(hipMemcpyAsync(c->h_txs.p, ftxs, sizeof(cg_filtered_tx) * n_ftx, hipMemcpyHostToDevice, s), "H2D ftxs");
  if (n_nodes)
    HIP_TRY(hipMemcpyAsync(c->h_comps.p, nodes, sizeof(cg_pmt_node) * n_nodes, hipMemcpyHostToDevice, s), "H2D nodes");
  if (n_leaves)
    HIP_TRY(hipMemcpyAsync(c->h_sigs.p, leaves, sizeof(cg_filtered_leaf) * n_leaves, hipMemcpyHostToDevice, s),
            "H2D leaves");
  if (arena_len) HIP_TRY(hipMemcpyAsync(c->arena.p, arena, arena_len, hipMemcpyHostToDevice, s), "H2D arena");
  HIP_TRY(cg::launch_filtered((const cg_filtered_tx*)c->h_txs.p, n_ftx, (const cg_pmt_node*)c->h_comps.p, n_nodes,
                              (const cg_filtered_leaf*)c->h_sigs.p, n_leaves, (const uint8_t*)c->arena.p, arena_len,
                              (uint8_t*)c->status.p, (uint8_t*)c->ftxws.p, s), "launch_filtered");
  HIP_TRY(hipMemcpyAsync(status_out, c->status.p, n_ftx, hipMemcpyDeviceToHost, s), "D2H status");
  HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
  return CG_OK;
}

}  // extern "C"
