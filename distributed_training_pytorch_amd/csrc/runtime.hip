// Native runtime pieces around the kernels:
//   * fine-grained/uncached device allocations + IPC handle export/import for
//     the xGMI exchange buffers (peer-mapped over xGMI),
//   * peer access management and peer copies (layer-split activations),
//   * a hipGraph step executor: captures `launches` back-to-back fused train
//     steps into ONE graph so a whole window of iterations costs one
//     hipGraphLaunch on the host (SURVEY.md §7.1 "capture the steady-state
//     iteration in a hipGraph").
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>

#include "dtp_api.h"

namespace {
thread_local std::string g_rt_err;
int rt_fail(hipError_t e, const char* what) {
  g_rt_err = std::string(what) + ": " + hipGetErrorString(e);
  return -(int)e - 1000;
}
#define RT_CHECK(x)                          \
  do {                                       \
    hipError_t _e = (x);                     \
    if (_e != hipSuccess) return rt_fail(_e, #x); \
  } while (0)

struct GraphHandle {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
};
}  // namespace

namespace dtp {
int set_err(int code, const char* msg) {
  g_rt_err = msg;
  return code;
}
int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_rt_err = std::string(what) + ": " + hipGetErrorString(e);
    return -3;
  }
  return 0;
}
}  // namespace dtp

extern "C" {

int dtp_version(void) { return 1; }

#ifndef DTP_SOURCE_HASH
#define DTP_SOURCE_HASH "unstamped"
#endif
// build stamp: build.py:source_hash() of the sources this library was compiled from
const char* dtp_source_hash(void) { return DTP_SOURCE_HASH; }
const char* dtp_last_error(void) { return g_rt_err.c_str(); }
const char* dtp_runtime_last_error(void) { return g_rt_err.c_str(); }

int dtp_get_device(int* dev) {
  RT_CHECK(hipGetDevice(dev));
  return 0;
}

int dtp_device_count(int* n) {
  RT_CHECK(hipGetDeviceCount(n));
  return 0;
}

int dtp_malloc_uncached(size_t bytes, void** out) {
  *out = nullptr;
  RT_CHECK(hipExtMallocWithFlags(out, bytes, hipDeviceMallocUncached));
  RT_CHECK(hipMemset(*out, 0, bytes));
  RT_CHECK(hipDeviceSynchronize());
  return 0;
}

int dtp_malloc(size_t bytes, void** out) {
  *out = nullptr;
  RT_CHECK(hipMalloc(out, bytes));
  RT_CHECK(hipMemset(*out, 0, bytes));
  RT_CHECK(hipDeviceSynchronize());
  return 0;
}

int dtp_free(void* p) {
  if (p) RT_CHECK(hipFree(p));
  return 0;
}

int dtp_ipc_handle_size(void) { return (int)sizeof(hipIpcMemHandle_t); }

int dtp_ipc_get_handle(void* p, void* out) {
  hipIpcMemHandle_t h;
  RT_CHECK(hipIpcGetMemHandle(&h, p));
  std::memcpy(out, &h, sizeof(h));
  return 0;
}

int dtp_ipc_open_handle(const void* handle, void** out) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  *out = nullptr;
  RT_CHECK(hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess));
  return 0;
}

int dtp_ipc_close_handle(void* p) {
  if (p) RT_CHECK(hipIpcCloseMemHandle(p));
  return 0;
}

int dtp_can_access_peer(int dev, int peer, int* out) {
  RT_CHECK(hipDeviceCanAccessPeer(out, dev, peer));
  return 0;
}

int dtp_enable_peer_access(int peer) {
  hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();
    return 0;
  }
  RT_CHECK(e);
  return 0;
}

int dtp_memcpy_peer_async(void* dst, int dst_dev, const void* src, int src_dev, size_t bytes, void* stream) {
  RT_CHECK(hipMemcpyPeerAsync(dst, dst_dev, src, src_dev, bytes, (hipStream_t)stream));
  return 0;
}

int dtp_memcpy_h2d(void* dst, const void* src, size_t bytes) {
  RT_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return 0;
}

int dtp_memcpy_d2h(void* dst, const void* src, size_t bytes) {
  RT_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return 0;
}

int dtp_stream_sync(void* stream) {
  RT_CHECK(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

// A stream whose kernels run only on the CUs set in `mask` (`words` 32-bit words,
// bit i = logical CU i).  The persistent train kernel is one workgroup per model:
// pinning its launches to the same few CUs keeps its code in those CUs' instruction
// cache from one launch to the next, instead of refetching it on whichever CUs the
// dispatcher picks (bench.py --cu-mask).
int dtp_stream_create_cu_mask(const unsigned* mask, int words, void** out) {
  *out = nullptr;
  if (!mask || words <= 0) return -1;
  hipStream_t s = nullptr;
  RT_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask));
  *out = s;
  return 0;
}

// A stream of the given priority (hipStreamCreateWithPriority; lower = higher priority).
// The layer-split engine's stages that share a GPU (persistent kernels that wait on each
// other) launch on streams of distinct priority levels: a hardware queue has one priority,
// so two such streams never sit in one in-order queue.  (Measured: CU-masked streams got
// separate queues yet ran one kernel after the other -- the second dispatch started when
// the first ended; profiles/r4_split_streams/.)
int dtp_stream_create_priority(int priority, void** out) {
  *out = nullptr;
  hipStream_t s = nullptr;
  RT_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority));
  *out = s;
  return 0;
}

int dtp_stream_priority_range(int* least, int* greatest) {
  RT_CHECK(hipDeviceGetStreamPriorityRange(least, greatest));
  return 0;
}

int dtp_stream_destroy(void* stream) {
  if (stream) RT_CHECK(hipStreamDestroy((hipStream_t)stream));
  return 0;
}

// debug mode (DTP_DEBUG=1): drain the device after a native call and surface any
// asynchronous kernel fault at the call that caused it
int dtp_device_sync_check(void) {
  RT_CHECK(hipDeviceSynchronize());
  RT_CHECK(hipGetLastError());
  return 0;
}

// ---- graph executor --------------------------------------------------------
int dtp_graph_capture_train(const DtpTrainArgs* a, int in, int h, int nl, int out, int mode, int launches,
                            void* stream, void** handle_out) {
  *handle_out = nullptr;
  if (launches <= 0) return -1;
  hipStream_t st = (hipStream_t)stream;
  auto* gh = new GraphHandle();
  hipError_t e = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) {
    delete gh;
    return rt_fail(e, "hipStreamBeginCapture");
  }
  int rc = 0;
  for (int i = 0; i < launches && rc == 0; ++i) rc = dtp_mlp_train(a, in, h, nl, out, mode, stream);
  e = hipStreamEndCapture(st, &gh->graph);
  if (rc != 0) {
    if (gh->graph) (void)hipGraphDestroy(gh->graph);
    delete gh;
    return rc;
  }
  if (e != hipSuccess) {
    delete gh;
    return rt_fail(e, "hipStreamEndCapture");
  }
  e = hipGraphInstantiate(&gh->exec, gh->graph, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    (void)hipGraphDestroy(gh->graph);
    delete gh;
    return rt_fail(e, "hipGraphInstantiate");
  }
  *handle_out = gh;
  return 0;
}

// `launches` one-step runs of a train engine (mlp_train.hip) captured into one graph;
// each run reads its step number from the device counters (host_t0 = -1), so every
// replay continues where the last one stopped
int dtp_train_engine_run(void* h, int n_steps, int t0, void* stream);
int dtp_graph_capture_engine(void* engine, int launches, void* stream, void** handle_out) {
  *handle_out = nullptr;
  if (launches <= 0 || !engine) return -1;
  hipStream_t st = (hipStream_t)stream;
  auto* gh = new GraphHandle();
  hipError_t e = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) {
    delete gh;
    return rt_fail(e, "hipStreamBeginCapture");
  }
  int rc = 0;
  for (int i = 0; i < launches && rc == 0; ++i) rc = dtp_train_engine_run(engine, 1, -1, stream);
  e = hipStreamEndCapture(st, &gh->graph);
  if (rc != 0) {
    if (gh->graph) (void)hipGraphDestroy(gh->graph);
    delete gh;
    return rc;
  }
  if (e != hipSuccess) {
    delete gh;
    return rt_fail(e, "hipStreamEndCapture");
  }
  e = hipGraphInstantiate(&gh->exec, gh->graph, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    (void)hipGraphDestroy(gh->graph);
    delete gh;
    return rt_fail(e, "hipGraphInstantiate");
  }
  *handle_out = gh;
  return 0;
}

int dtp_graph_launch(void* handle, void* stream) {
  auto* gh = static_cast<GraphHandle*>(handle);
  if (!gh) return -1;
  RT_CHECK(hipGraphLaunch(gh->exec, (hipStream_t)stream));
  return 0;
}

int dtp_graph_destroy(void* handle) {
  auto* gh = static_cast<GraphHandle*>(handle);
  if (!gh) return 0;
  if (gh->exec) (void)hipGraphExecDestroy(gh->exec);
  if (gh->graph) (void)hipGraphDestroy(gh->graph);
  delete gh;
  return 0;
}

}  // extern "C"

// ABI guard: _native.py compares these with its ctypes mirrors at load time
extern "C" int dtp_struct_sizes(int* out) {
  out[0] = (int)sizeof(dtp::SamplerCfg);
  out[1] = (int)sizeof(DtpHyper);
  out[2] = (int)sizeof(DtpTrainArgs);
  out[3] = (int)sizeof(DtpStageArgs);
  out[4] = (int)sizeof(DtpOptArgs);
  out[5] = (int)sizeof(DtpGemmArgs);
  out[6] = (int)sizeof(DtpSplitStageArgs);
  out[7] = (int)sizeof(DtpSplitLaunch);
  return 8;
}
