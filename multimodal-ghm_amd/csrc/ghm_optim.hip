// clip_grad_norm_ + custom AdamW over the flat fp32 parameter/gradient buffers.
// Reference: train_CLIP.py:163-167, models/optimizer.py:41-85.  The AdamW update
// uses explicitly rounded IEEE ops (no FMA contraction), in the reference's
// operation order, so given identical gradients the parameters match a PyTorch
// CPU run bit for bit.
#include <string.h>

#include "ghm_common.h"
#include "ghm_launch.h"

static thread_local char g_err[512] = "";

void ghm_set_error(const char* msg, const char* file, int line) {
  snprintf(g_err, sizeof(g_err), "%s (%s:%d)", msg, file, line);
}

extern "C" const char* ghm_last_error_string(void) { return g_err; }

int ghm_launch_status() {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "HIP launch failed: %s", hipGetErrorString(e));
    return static_cast<int>(e);
  }
  return GHM_OK;
}

extern "C" int64_t ghm_token_blocks(int64_t M) { return (M + 127) / 128; }

extern "C" int ghm_device_ok(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  return strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

// Cross-stream ordering for the two-tower step (clip_trainer.py _phase /
// _cross_wait): events recorded with a device-scope release instead of the
// default system-scope one (mode 1: hipEventReleaseToDevice; 2:
// hipEventDisableSystemFence; HIP takes one release flag) -- the waits order work
// on one device, no host or peer reads the data.
extern "C" void* ghm_event_create(int mode) {
  hipEvent_t e = nullptr;
  const unsigned flags = hipEventDisableTiming | (mode == 1 ? hipEventReleaseToDevice
                                                  : mode == 2 ? hipEventDisableSystemFence : 0u);
  const hipError_t rc = hipEventCreateWithFlags(&e, flags);
  if (rc != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "hipEventCreateWithFlags(0x%x): %s", flags, hipGetErrorString(rc));
    return nullptr;
  }
  return e;
}

extern "C" int ghm_event_destroy(void* ev) {
  GHM_CHECK(ev, "null event");
  return hipEventDestroy(static_cast<hipEvent_t>(ev)) == hipSuccess ? GHM_OK : -1;
}

extern "C" int ghm_event_record(void* ev, void* stream) {
  GHM_CHECK(ev, "null event");
  if (hipEventRecord(static_cast<hipEvent_t>(ev), ghm_stream(stream)) != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "hipEventRecord failed");
    return -1;
  }
  return GHM_OK;
}

extern "C" int ghm_stream_wait(void* stream, void* ev) {
  GHM_CHECK(ev, "null event");
  if (hipStreamWaitEvent(ghm_stream(stream), static_cast<hipEvent_t>(ev), 0) != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "hipStreamWaitEvent failed");
    return -1;
  }
  return GHM_OK;
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_sumsq(const float* __restrict__ g, int64_t n,
                                               float* __restrict__ part) {
  __shared__ float red[4];
  float acc = 0.f;
  const int64_t n4 = n / 4;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n4;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const float4 v = g4[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const float v = g[n4 * 4 + threadIdx.x];
    acc += v * v;
  }
  acc = sum32(acc);
  acc += __shfl_xor(acc, 32, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void k_clip_finalize(const float* __restrict__ part, int nparts,
                                                       float max_norm, const float* __restrict__ sched,
                                                       int n_sched, int32_t* __restrict__ step,
                                                       float* __restrict__ hyper) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) acc += part[i];
  acc = sum32(acc);
  acc += __shfl_xor(acc, 32, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float norm = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
    float coef = max_norm / (norm + 1e-6f);  // torch clip_grad_norm_
    coef = coef < 1.f ? coef : 1.f;
    hyper[0] = norm;
    hyper[1] = coef;
    int s = *step;
    const int si = s < n_sched ? s : n_sched - 1;
    hyper[2] = sched[2 * si];
    hyper[3] = sched[2 * si + 1];
    *step = s + 1;
  }
}

__global__ __launch_bounds__(256) void k_adamw(float* __restrict__ p, const float* __restrict__ g,
                                               float* __restrict__ m, float* __restrict__ v, int64_t n,
                                               const float* __restrict__ hyper, float b1, float omb1,
                                               float b2, float omb2, float eps) {
  const float coef = hyper[1], lr_t = hyper[2], lr_wd = hyper[3];
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const float gg = __fmul_rn(g[i], coef);                                       // grads *= clip_coef
    const float mm = __fadd_rn(__fmul_rn(b1, m[i]), __fmul_rn(omb1, gg));         // beta1*m + (1-beta1)*g
    const float vv = __fadd_rn(__fmul_rn(b2, v[i]), __fmul_rn(omb2, __fmul_rn(gg, gg)));
    // sqrt and divide evaluated in f64 and rounded once to f32: correctly rounded
    // f32 results (53 >= 2*24 + 2), unlike the f32 hardware sequences.
    const float sq = static_cast<float>(sqrt(static_cast<double>(vv)));
    const float upd = static_cast<float>(static_cast<double>(__fmul_rn(lr_t, mm)) /
                                         static_cast<double>(__fadd_rn(sq, eps)));
    float pp = __fsub_rn(p[i], upd);                                              // p -= lr_t m/(sqrt v+eps)
    pp = __fsub_rn(pp, __fmul_rn(lr_wd, pp));                                     // p -= lr*wd*p
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

extern "C" int ghm_clip_prepare(const float* grad, int64_t n, float max_norm, const float* sched,
                                int n_sched, int32_t* step, float* hyper, float* work, void* stream) {
  GHM_CHECK(grad && sched && step && hyper && work, "null pointer");
  GHM_CHECK(n >= 1 && n_sched >= 1, "shape");
  const int nb = 1024;
  hipStream_t s = ghm_stream(stream);
  hipLaunchKernelGGL(k_sumsq, dim3(nb), dim3(256), 0, s, grad, n, work);
  int st = ghm_launch_status();
  if (st) return st;
  hipLaunchKernelGGL(k_clip_finalize, dim3(1), dim3(256), 0, s, work, nb, max_norm, sched, n_sched, step, hyper);
  return ghm_launch_status();
}

extern "C" int ghm_adamw(float* param, const float* grad, float* m, float* v, int64_t n,
                         const float* hyper, float b1, float one_minus_b1, float b2, float one_minus_b2,
                         float eps, void* stream) {
  GHM_CHECK(param && grad && m && v && hyper, "null pointer");
  GHM_CHECK(n >= 1, "shape");
  int64_t nb = (n + 255) / 256;
  if (nb > 2048) nb = 2048;
  hipLaunchKernelGGL(k_adamw, dim3(static_cast<unsigned>(nb)), dim3(256), 0, ghm_stream(stream), param, grad, m,
                     v, n, hyper, b1, one_minus_b1, b2, one_minus_b2, eps);
  return ghm_launch_status();
}
