// libhnm_mi355x: context, errors, workspace, and the small memory-bound kernels
// (row gather, layer-1 projection, axpby, top-K merge).
#include <stdlib.h>
#include <string.h>

#include "hnm_device.h"
#include "hnm_internal.h"

static thread_local char g_err[512] = "";

void hnm_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" int hnm_abi_version(void) { return HNM_ABI_VERSION; }
extern "C" const char* hnm_last_error(void) { return g_err; }

extern "C" hnm_status hnm_ctx_create(int device, hnm_ctx** out) {
  HNM_REQUIRE(out, HNM_EINVAL, "hnm_ctx_create: out is NULL");
  int ndev = 0;
  HNM_HIP_CHECK(hipGetDeviceCount(&ndev));
  HNM_REQUIRE(device >= 0 && device < ndev, HNM_EINVAL, "hnm_ctx_create: no device %d (%d visible)",
              device, ndev);
  const HnmDeviceGuard guard(device);  // the caller's current device is restored on return
  hnm_ctx* c = (hnm_ctx*)calloc(1, sizeof(hnm_ctx));
  HNM_REQUIRE(c, HNM_ENOMEM, "hnm_ctx_create: out of host memory");
  c->device = device;
  c->stream = 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->num_cus = prop.multiProcessorCount;
  if (c->num_cus <= 0) c->num_cus = 256;
  c->prefilter = 1;
  c->strided = 0;
  c->deep_mfma = 1;
#ifndef HNM_LINEAR_MFMA_DEFAULT  // A/B builds only (tools/build_variant.sh)
#define HNM_LINEAR_MFMA_DEFAULT 1
#endif
  c->linear_mfma = HNM_LINEAR_MFMA_DEFAULT;
  if (hipMalloc((void**)&c->err_dev, 64) != hipSuccess) {
    free(c);
    hnm_set_error("hnm_ctx_create: hipMalloc of the error word failed");
    return HNM_ENOMEM;
  }
  HNM_HIP_CHECK(hipMemset(c->err_dev, 0, 64));
  HNM_HIP_CHECK(hipEventCreateWithFlags(&c->chain_ev, hipEventDisableTiming));
  HNM_HIP_CHECK(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
  HNM_HIP_CHECK(hipEventCreateWithFlags(&c->side_in, hipEventDisableTiming));
  HNM_HIP_CHECK(hipEventCreateWithFlags(&c->side_out, hipEventDisableTiming));
  // counters of the certified pre-filter live in the same allocation (8-byte aligned)
  c->stats_dev = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(c->err_dev) + 8);
  *out = c;
  return HNM_OK;
}

extern "C" hnm_status hnm_ctx_destroy(hnm_ctx* ctx) {
  HNM_CTX_DEVICE(ctx);
  if (!ctx) return HNM_OK;
  (void)hipDeviceSynchronize();
  for (int i = 0; i < ctx->cap; ++i) {
    (void)hipEventDestroy(ctx->ev0[i]);
    (void)hipEventDestroy(ctx->ev1[i]);
  }
  free(ctx->ev0);
  free(ctx->ev1);
  hnm_rccl_release(ctx);
  if (ctx->ws) (void)hipFree(ctx->ws);
  if (ctx->err_dev) (void)hipFree(ctx->err_dev);
  (void)hipEventDestroy(ctx->chain_ev);
  (void)hipEventDestroy(ctx->side_in);
  (void)hipEventDestroy(ctx->side_out);
  (void)hipStreamDestroy(ctx->side);
  free(ctx);
  return HNM_OK;
}

extern "C" hnm_status hnm_ctx_set_stream(hnm_ctx* ctx, void* s) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx, HNM_EINVAL, "ctx is NULL");
  const hipStream_t ns = (hipStream_t)s;
  if (ns == ctx->stream) return HNM_OK;
  // The workspace and the two-phase tables are shared by every call on this ctx: queue the
  // new stream behind everything already issued on the old one (no host sync).
  HNM_HIP_CHECK(hipEventRecord(ctx->chain_ev, ctx->stream));
  HNM_HIP_CHECK(hipStreamWaitEvent(ns, ctx->chain_ev, 0));
  ctx->stream = ns;
  return HNM_OK;
}

extern "C" hnm_status hnm_ctx_abort_pending(hnm_ctx* ctx) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx, HNM_EINVAL, "ctx is NULL");
  ctx->pend.kind = 0;
  return HNM_OK;
}

extern "C" hnm_status hnm_ctx_set_option(hnm_ctx* ctx, int option, int64_t value) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx, HNM_EINVAL, "ctx is NULL");
  switch (option) {
    case HNM_OPT_PREFILTER:
      ctx->prefilter = value != 0;
      return HNM_OK;
    case HNM_OPT_STATS:
      ctx->stats_on = value != 0;
      return HNM_OK;
    case HNM_OPT_STRIDED:
      ctx->strided = value != 0;
      return HNM_OK;
    case HNM_OPT_DEEP_MFMA:
      ctx->deep_mfma = value != 0;
      return HNM_OK;
    case HNM_OPT_LINEAR_MFMA:
      ctx->linear_mfma = value != 0;
      return HNM_OK;
    default:
      hnm_set_error("hnm_ctx_set_option: unknown option %d", option);
      return HNM_EINVAL;
  }
}

extern "C" hnm_status hnm_ctx_prefilter_stats(hnm_ctx* ctx, int64_t* out, int reset) {
  HNM_CTX_DEVICE(ctx);
  return hnm_ctx_prefilter_stats_ex(ctx, out, 3, reset);
}

extern "C" hnm_status hnm_ctx_prefilter_stats_ex(hnm_ctx* ctx, int64_t* out, int n, int reset) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && out, HNM_EINVAL, "ctx/out is NULL");
  HNM_REQUIRE(n >= 1 && n <= HNM_STATS_N, HNM_EINVAL, "prefilter_stats: 1 <= n <= %d", HNM_STATS_N);
  // device-wide sync: never reads ctx->stream, which the ctx's owning thread may be switching
  // (this entry is called across threads: the Python layer sums every thread's ctx).  The
  // calling thread's current device is restored on every exit path.
  int prev = -1;
  HNM_HIP_CHECK(hipGetDevice(&prev));
  struct Restore {
    int dev;
    ~Restore() { (void)hipSetDevice(dev); }
  } restore{prev};
  HNM_HIP_CHECK(hipSetDevice(ctx->device));
  HNM_HIP_CHECK(hipDeviceSynchronize());
  unsigned long long v[HNM_STATS_N];
  HNM_HIP_CHECK(hipMemcpy(v, ctx->stats_dev, sizeof(v), hipMemcpyDeviceToHost));
  for (int i = 0; i < n; ++i) out[i] = (int64_t)v[i];
  if (reset) HNM_HIP_CHECK(hipMemset(ctx->stats_dev, 0, sizeof(v)));
  return HNM_OK;
}

extern "C" hnm_status hnm_ctx_num_cus(hnm_ctx* ctx, int* out) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && out, HNM_EINVAL, "ctx/out is NULL");
  *out = ctx->num_cus;
  return HNM_OK;
}

hnm_status hnm_workspace(hnm_ctx* ctx, size_t bytes, void** out) {
  HNM_REQUIRE(!ctx->pend.kind, HNM_EINVAL,
              "a two-phase top-K call is open on this ctx: call its _finish first");
  bytes = hnm_align(bytes);
  if (bytes > ctx->ws_size) {
    HNM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    if (ctx->ws) HNM_HIP_CHECK(hipFree(ctx->ws));
    ctx->ws = nullptr;
    ctx->ws_size = 0;
    size_t want = hnm_align(bytes + bytes / 4);
    if (hipMalloc(&ctx->ws, want) != hipSuccess) {
      hnm_set_error("workspace: hipMalloc(%zu) failed", want);
      return HNM_ENOMEM;
    }
    ctx->ws_size = want;
  }
  *out = ctx->ws;
  return HNM_OK;
}

__global__ void fill_f32_kernel(float* __restrict__ p, int64_t n, float v) {
  const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (x < n) p[x] = v;
}

hnm_status hnm_fill_f32(hnm_ctx* ctx, float* p, int64_t n, float v) {
  if (n <= 0) return HNM_OK;
  hipLaunchKernelGGL(fill_f32_kernel, dim3((unsigned)hnm_cdiv(n, 256)), dim3(256), 0, ctx->stream,
                     p, n, v);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

extern "C" hnm_status hnm_ctx_reserve(hnm_ctx* ctx, size_t bytes) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx, HNM_EINVAL, "ctx is NULL");
  void* p;
  return hnm_workspace(ctx, bytes, &p);
}

// ------------------------------------------------------------------ kernel timer
#define HNM_TIMER_PREALLOC 1024
static bool timer_grow(hnm_ctx* ctx, int ncap) {
  hipEvent_t* a = (hipEvent_t*)realloc(ctx->ev0, ncap * sizeof(hipEvent_t));
  if (a) ctx->ev0 = a;
  hipEvent_t* b = (hipEvent_t*)realloc(ctx->ev1, ncap * sizeof(hipEvent_t));
  if (b) ctx->ev1 = b;
  if (!a || !b) return false;
  for (int i = ctx->cap; i < ncap; ++i) {
    (void)hipEventCreate(&ctx->ev0[i]);
    (void)hipEventCreate(&ctx->ev1[i]);
  }
  ctx->cap = ncap;
  return true;
}

void hnm_timer_begin(hnm_ctx* ctx, int cls) {
  if (!(ctx->timing & cls)) return;
  if (ctx->nev == ctx->cap && !timer_grow(ctx, ctx->cap ? 2 * ctx->cap : 256)) {
    ctx->timing = 0;
    return;
  }
  (void)hipEventRecord(ctx->ev0[ctx->nev], ctx->stream);
}

void hnm_timer_end(hnm_ctx* ctx, int cls) {
  if (!(ctx->timing & cls) || ctx->nev >= ctx->cap) return;
  (void)hipEventRecord(ctx->ev1[ctx->nev], ctx->stream);
  ++ctx->nev;
}

extern "C" hnm_status hnm_ctx_enable_timing(hnm_ctx* ctx, int on) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx, HNM_EINVAL, "ctx is NULL");
  // the events are created here, outside the caller's timed region (a bench loop of a few
  // hundred launches records into them without creating any)
  if (on && ctx->cap < HNM_TIMER_PREALLOC && !timer_grow(ctx, HNM_TIMER_PREALLOC)) on = 0;
  ctx->timing = on;
  ctx->nev = 0;
  return HNM_OK;
}

extern "C" hnm_status hnm_ctx_timing(hnm_ctx* ctx, double* total_ms, int64_t* launches) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && total_ms && launches, HNM_EINVAL, "hnm_ctx_timing: NULL argument");
  HNM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  double t = 0.0;
  for (int i = 0; i < ctx->nev; ++i) {
    float ms = 0.f;
    HNM_HIP_CHECK(hipEventElapsedTime(&ms, ctx->ev0[i], ctx->ev1[i]));
    t += ms;
  }
  *total_ms = t;
  *launches = ctx->nev;
  ctx->nev = 0;
  return HNM_OK;
}

extern "C" hnm_status hnm_ctx_check(hnm_ctx* ctx) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx, HNM_EINVAL, "ctx is NULL");
  unsigned h = 0;
  HNM_HIP_CHECK(hipMemcpyAsync(&h, ctx->err_dev, sizeof(unsigned), hipMemcpyDeviceToHost,
                               ctx->stream));
  HNM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  if (h) {
    HNM_HIP_CHECK(hipMemsetAsync(ctx->err_dev, 0, sizeof(unsigned), ctx->stream));
    if (h & HNM_ERR_OOB) {
      hnm_set_error("index out of range in self (an id exceeded the embedding table)");
      return HNM_EOOB;
    }
    if (h & HNM_ERR_MASK_CAP) {
      hnm_set_error("hnm_mask_gather_csr: the batch's history ids exceeded the mask capacity "
                    "(rows were truncated)");
      return HNM_EINVAL;
    }
  }
  return HNM_OK;
}

// ------------------------------------------------------------------ a1 gather
// One wave per output row; float4 lanes when rows are 16-B aligned.
__global__ __launch_bounds__(256) void gather_rows_kernel(const float* __restrict__ tab,
                                                          int64_t rows, int64_t ld, int d,
                                                          const int64_t* __restrict__ ids,
                                                          int64_t n, float* __restrict__ out,
                                                          int64_t ldo, unsigned* err,
                                                          bool vec4) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const int lane = threadIdx.x & 63;
  const int64_t id = ids[r];
  float* o = out + r * ldo;
  if (id < 0 || id >= rows) {
    if (lane == 0) hnm_flag(err, HNM_ERR_OOB);
    for (int c = lane; c < d; c += 64) o[c] = __builtin_nanf("");
    return;
  }
  const float* src = tab + id * ld;
  if (vec4) {
    for (int c = lane * 4; c < d; c += 256)
      *reinterpret_cast<float4*>(o + c) = *reinterpret_cast<const float4*>(src + c);
  } else {
    for (int c = lane; c < d; c += 64) o[c] = src[c];
  }
}

extern "C" hnm_status hnm_gather_rows_f32(hnm_ctx* ctx, const float* table, int64_t rows,
                                          int64_t ld, int d, const int64_t* ids, int64_t n,
                                          float* out, int64_t ldo) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && table && ((ids && out) || n == 0), HNM_EINVAL, "gather: NULL argument");
  HNM_REQUIRE(d > 0 && ld >= d && ldo >= d && rows > 0, HNM_EINVAL, "gather: bad shape");
  if (n <= 0) return HNM_OK;
  const bool vec4 = (d % 4 == 0) && (ld % 4 == 0) && (ldo % 4 == 0) &&
                    ((uintptr_t)table % 16 == 0) && ((uintptr_t)out % 16 == 0);
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)hnm_cdiv(n, 4)), dim3(256), 0,
                     ctx->stream, table, rows, ld, d, ids, n, out, ldo, ctx->err_dev, vec4);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

// ------------------------------------------------------------------ projection
// Y[r, c(n)] = sum_k X[x(r), k] W[n, k] (+ b[n]).  TM rows x 64 outputs per block (TM = 64,
// or 16 for short inputs -- a batch of users -- so the grid still covers the CUs), K in
// chunks of 32 staged through LDS; each thread owns a TM/16 x 4 output patch.  fp32 FMA
// chain in k order whatever TM (a per-item / per-user precompute: <1 % of any scoring kernel).
#define LIN_TN 64
#define LIN_TK 32
// VEC (K, ldx, ldw multiples of 4, 16-B aligned X and W): 16-B global loads, and the compute
// loop reads its x / w operands as float4 from the 16-B-aligned LDS rows (2 LDS reads per 16
// FMAs instead of 8); the FMA chain per output is the same k-ordered one either way.
template <int LIN_TM, bool VEC>
__global__ __launch_bounds__(256) void linear_rows_kernel(
    const float* __restrict__ X, int64_t ldx, const int64_t* __restrict__ ids, int64_t x_rows,
    int64_t M, int K, const float* __restrict__ W, int64_t ldw, const float* __restrict__ bias,
    int N, float* __restrict__ Y, int64_t ldy, int pair_permute, unsigned* err) {
  constexpr int RPT = LIN_TM / 16;  // rows per thread
  constexpr int XP = LIN_TM + (VEC ? 4 : 1), WP = LIN_TN + (VEC ? 4 : 1);
  __shared__ __attribute__((aligned(16))) float xs[LIN_TK][XP];
  __shared__ __attribute__((aligned(16))) float ws[LIN_TK][WP];
  const int t = threadIdx.x;
  const int64_t m0 = (int64_t)blockIdx.x * LIN_TM;
  const int n0 = blockIdx.y * LIN_TN;
  const int tr = (t >> 4) * RPT;  // rows tr..tr+RPT-1
  const int tc = (t & 15) * 4;    // cols tc..tc+3
  float acc[RPT][4] = {};
  for (int k0 = 0; k0 < K; k0 += LIN_TK) {
    if (VEC) {
      for (int e = t; e < LIN_TM * LIN_TK / 4; e += 256) {
        const int rr = e / (LIN_TK / 4), kq = 4 * (e % (LIN_TK / 4));
        const int64_t m = m0 + rr;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (m < M && k0 + kq < K) {
          const int64_t src = ids ? ids[m] : m;
          if (src < 0 || src >= x_rows) {
            if (kq == 0) hnm_flag(err, HNM_ERR_OOB);
            v = make_float4(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""),
                            __builtin_nanf(""));
          } else {
            v = *reinterpret_cast<const float4*>(X + src * ldx + k0 + kq);
          }
        }
        xs[kq][rr] = v.x;
        xs[kq + 1][rr] = v.y;
        xs[kq + 2][rr] = v.z;
        xs[kq + 3][rr] = v.w;
      }
      for (int e = t; e < LIN_TN * LIN_TK / 4; e += 256) {
        const int nn = e / (LIN_TK / 4), kq = 4 * (e % (LIN_TK / 4));
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (n0 + nn < N && k0 + kq < K)
          v = *reinterpret_cast<const float4*>(W + (int64_t)(n0 + nn) * ldw + k0 + kq);
        ws[kq][nn] = v.x;
        ws[kq + 1][nn] = v.y;
        ws[kq + 2][nn] = v.z;
        ws[kq + 3][nn] = v.w;
      }
    } else {
      for (int e = t; e < LIN_TM * LIN_TK; e += 256) {
        const int rr = e / LIN_TK, kk = e % LIN_TK;
        const int64_t m = m0 + rr;
        float v = 0.f;
        if (m < M && k0 + kk < K) {
          int64_t src = ids ? ids[m] : m;
          if (src < 0 || src >= x_rows) {
            if (kk == 0) hnm_flag(err, HNM_ERR_OOB);
            v = __builtin_nanf("");
          } else {
            v = X[src * ldx + k0 + kk];
          }
        }
        xs[kk][rr] = v;
      }
      for (int e = t; e < LIN_TN * LIN_TK; e += 256) {
        const int nn = e / LIN_TK, kk = e % LIN_TK;
        float v = 0.f;
        if (n0 + nn < N && k0 + kk < K) v = W[(int64_t)(n0 + nn) * ldw + k0 + kk];
        ws[kk][nn] = v;
      }
    }
    __syncthreads();
    const int kmax = min(LIN_TK, K - k0);
    for (int kk = 0; kk < kmax; ++kk) {
      float xv[RPT], wv[4];
      if (VEC && RPT == 4) {
        const float4 a = *reinterpret_cast<const float4*>(&xs[kk][tr]);
        xv[0] = a.x; xv[RPT > 1 ? 1 : 0] = a.y; xv[RPT > 2 ? 2 : 0] = a.z; xv[RPT > 3 ? 3 : 0] = a.w;
      } else {
#pragma unroll
        for (int i = 0; i < RPT; ++i) xv[i] = xs[kk][tr + i];
      }
      if (VEC) {
        const float4 b = *reinterpret_cast<const float4*>(&ws[kk][tc]);
        wv[0] = b.x; wv[1] = b.y; wv[2] = b.z; wv[3] = b.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) wv[j] = ws[kk][tc + j];
      }
#pragma unroll
      for (int i = 0; i < RPT; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(xv[i], wv[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int64_t m = m0 + tr + i;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tc + j;
      if (n >= N) continue;
      float v = acc[i][j];
      if (bias) v += bias[n];
      const int64_t c = pair_permute ? (int64_t)(n & 1) * (ldy / 2) + (n >> 1) : n;
      Y[m * ldy + c] = v;
    }
  }
}

// Round 6: the same projection on the fp32 matrix pipe when K is a multiple of 32 (the NCF
// and W&D layer-1 halves: K = h0 / d = 64).  v_mfma_f32_32x32x2_f32 is an exact fp32 fma chain
// in k order (tools/mfma_semantics_probe.hip (a)), so a chain of them from C = 0 over k = 0, 1,
// .., K-1 and the bias added after is bitwise linear_rows_kernel's per-output fmaf chain
// (tests/test_gpu_abi_rows.py checks both kernels on the same inputs).  64 rows x 64 outputs a
// block, one 32 x 32 output tile a wave (waves 2 r + c: rows 32 r, outputs 32 c), K in chunks
// of 32 staged through LDS as in linear_rows_kernel (16-B global loads).  rocprofv3 minima
// (profiles/r10g_linear_rows_ab.txt): NCF's item half (105,542 x 64 x 64) 21.0 -> 18.1 us,
// W&D's (105,542 x 512 x 64) 115.2 -> 100.5 us -- the staging, not the FMAs, bounds both.
__global__ __launch_bounds__(256) void linear_rows_mfma_kernel(
    const float* __restrict__ X, int64_t ldx, const int64_t* __restrict__ ids, int64_t x_rows,
    int64_t M, int K, const float* __restrict__ W, int64_t ldw, const float* __restrict__ bias,
    int N, float* __restrict__ Y, int64_t ldy, int pair_permute, unsigned* err) {
  constexpr int RS = LIN_TK + 1;  // LDS row stride (floats): rows spread over the banks
  __shared__ float xs[64 * RS];   // [row][k] of the chunk
  __shared__ float ws[64 * RS];   // [output][k]
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int64_t m0 = (int64_t)blockIdx.x * 64;
  const int n0 = blockIdx.y * LIN_TN;
  const int wr = 32 * (wave >> 1), wc = 32 * (wave & 1);
  f32x16 acc = {};
  for (int k0 = 0; k0 < K; k0 += LIN_TK) {
    for (int e = t; e < 64 * LIN_TK / 4; e += 256) {
      const int rr = e / (LIN_TK / 4), kq = 4 * (e % (LIN_TK / 4));
      const int64_t m = m0 + rr;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < M) {
        const int64_t src = ids ? ids[m] : m;
        if (src < 0 || src >= x_rows) {
          if (kq == 0) hnm_flag(err, HNM_ERR_OOB);
          v = make_float4(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""),
                          __builtin_nanf(""));
        } else {
          v = *reinterpret_cast<const float4*>(X + src * ldx + k0 + kq);
        }
      }
      float* xr = xs + rr * RS + kq;
      xr[0] = v.x; xr[1] = v.y; xr[2] = v.z; xr[3] = v.w;
    }
    for (int e = t; e < LIN_TN * LIN_TK / 4; e += 256) {
      const int nn = e / (LIN_TK / 4), kq = 4 * (e % (LIN_TK / 4));
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (n0 + nn < N) v = *reinterpret_cast<const float4*>(W + (int64_t)(n0 + nn) * ldw + k0 + kq);
      float* wr4 = ws + nn * RS + kq;
      wr4[0] = v.x; wr4[1] = v.y; wr4[2] = v.z; wr4[3] = v.w;
    }
    __syncthreads();
    const float* xa = xs + (wr + i) * RS + h;  // A[i][h] of step s: row wr + i, k = 2 s + h
    const float* wb = ws + (wc + i) * RS + h;  // B[h][j = i]: output wc + i, k = 2 s + h
#pragma unroll
    for (int st = 0; st < LIN_TK / 2; ++st) acc = mfma32x32x2(xa[2 * st], wb[2 * st], acc);
    __syncthreads();
  }
  const int n = n0 + wc + i;
  if (n >= N) return;
  const float bn = bias ? bias[n] : 0.f;
  const int64_t c = pair_permute ? (int64_t)(n & 1) * (ldy / 2) + (n >> 1) : n;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t m = m0 + wr + mfma32_row(r, h);
    if (m >= M) continue;
    float v = acc[r];
    if (bias) v += bn;
    Y[m * ldy + c] = v;
  }
}

extern "C" hnm_status hnm_linear_rows_f32(hnm_ctx* ctx, const float* X, int64_t ldx,
                                          const int64_t* ids, int64_t x_rows, int64_t M, int K,
                                          const float* W, int64_t ldw, const float* bias, int N,
                                          float* Y, int64_t ldy, int pair_permute) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && X && W && Y, HNM_EINVAL, "linear_rows: NULL argument");
  HNM_REQUIRE(K > 0 && N > 0 && ldx >= K && ldw >= K && ldy >= N, HNM_EINVAL,
              "linear_rows: bad shape");
  HNM_REQUIRE(!pair_permute || (ldy % 2 == 0 && N <= ldy), HNM_EINVAL,
              "linear_rows: pair_permute needs an even ldy");
  if (M <= 0) return HNM_OK;
  const bool short_in = hnm_cdiv(M, 64) < 2 * (int64_t)ctx->num_cus;
  const int tm = short_in ? 16 : 64;
  const bool vec = K % 4 == 0 && ldx % 4 == 0 && ldw % 4 == 0 && ((uintptr_t)X & 15) == 0 &&
                   ((uintptr_t)W & 15) == 0;
  if (vec && K % LIN_TK == 0 && !short_in && ctx->linear_mfma) {
    hipLaunchKernelGGL(linear_rows_mfma_kernel, dim3((unsigned)hnm_cdiv(M, 64), (unsigned)hnm_cdiv(N, LIN_TN)),
                       dim3(256), 0, ctx->stream, X, ldx, ids, ids ? x_rows : M, M, K, W, ldw, bias,
                       N, Y, ldy, pair_permute, ctx->err_dev);
    HNM_LAUNCH_CHECK();
    return HNM_OK;
  }
  dim3 grid((unsigned)hnm_cdiv(M, tm), (unsigned)hnm_cdiv(N, LIN_TN));
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, ctx->stream, X, ldx, ids, ids ? x_rows : M, M,
                       K, W, ldw, bias, N, Y, ldy, pair_permute, ctx->err_dev);
  };
  if (short_in) vec ? launch(linear_rows_kernel<16, true>) : launch(linear_rows_kernel<16, false>);
  else vec ? launch(linear_rows_kernel<64, true>) : launch(linear_rows_kernel<64, false>);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

// ------------------------------------------------------------------ axpby
__global__ __launch_bounds__(256) void axpby_kernel(int64_t n, float a, const float* __restrict__ x,
                                                    float b, const float* __restrict__ y,
                                                    float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    float v = a * x[i];
    if (y) v += b * y[i];
    out[i] = v;
  }
}

extern "C" hnm_status hnm_axpby_f32(hnm_ctx* ctx, int64_t n, float alpha, const float* x,
                                    float beta, const float* y, float* out) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && ((x && out) || n == 0), HNM_EINVAL, "axpby: NULL argument");
  if (n <= 0) return HNM_OK;
  const unsigned grid = (unsigned)std::min<int64_t>(hnm_cdiv(n, 256), 8 * 2048);
  hipLaunchKernelGGL(axpby_kernel, dim3(grid), dim3(256), 0, ctx->stream, n, alpha, x, beta,
                     y, out);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

// ------------------------------------------------------------------ top-K merge
// One wave per row: candidates stream through the wave list 64 at a time.
// rows/nrows (optional): candidate row b is output row rows[b], for b < *nrows.
template <int NS, typename IdxT>
__global__ __launch_bounds__(256) void topk_merge_kernel(const float* __restrict__ cv,
                                                         const IdxT* __restrict__ ci, int64_t B,
                                                         int64_t G, int64_t gstride,
                                                         int64_t bstride, int kc, int k,
                                                         float* __restrict__ ov,
                                                         int64_t* __restrict__ oi,
                                                         const int32_t* __restrict__ rows,
                                                         const int32_t* __restrict__ nrows,
                                                         int64_t dyn_items, int dyn_cus) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nb = nrows ? (int64_t)*nrows : B;
  if (b >= nb) return;
  if (dyn_cus > 0) {  // row-list candidates: np partitions per row, as the launch chose them
    kc *= choose_partition(dyn_items, hnm_cdiv(nb, 128), dyn_cus).np;
    bstride = kc;
  }
  const int64_t ob = rows ? (int64_t)rows[b] : b;
  const int lane = threadIdx.x & 63;
  WaveTopK<NS> L;
  L.init();
  const int64_t n = G * (int64_t)kc;
  // 4 chunks of 64 candidates per round, every load issued before the first offer (one load
  // round trip per chunk made a row-list merge of ~5.6k candidates a row latency-bound)
  constexpr int U = 4;
  for (int64_t base = 0; base < n; base += 64 * U) {
    IdxT ii[U];
    float vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = base + 64 * u + lane;
      ii[u] = -1;
      vv[u] = -__builtin_inff();
      if (j < n) {
        const int64_t g = j / kc, q = j % kc;
        const int64_t off = g * gstride + b * bstride + q;
        ii[u] = ci[off];
        vv[u] = cv[off];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = ii[u] >= 0;
      L.offer(ok ? vv[u] : -__builtin_inff(), ok ? (int)ii[u] : HNM_SENTINEL_IDX, ok, k);
    }
  }
  L.store(ov ? ov + ob * k : nullptr, oi + ob * k, k);
}

template <typename IdxT>
hnm_status launch_merge(hnm_ctx* ctx, const float* cv, const IdxT* ci, int64_t B, int64_t G,
                        int64_t gstride, int64_t bstride, int kc, int k, float* ov,
                        int64_t* oi, const int32_t* rows = nullptr,
                        const int32_t* nrows = nullptr, int64_t dyn_items = 0, int dyn_cus = 0) {
  dim3 grid((unsigned)hnm_cdiv(B, 4));
  if (k <= 64)
    hipLaunchKernelGGL((topk_merge_kernel<1, IdxT>), grid, dim3(256), 0, ctx->stream, cv, ci,
                       B, G, gstride, bstride, kc, k, ov, oi, rows, nrows, dyn_items, dyn_cus);
  else
    hipLaunchKernelGGL((topk_merge_kernel<2, IdxT>), grid, dim3(256), 0, ctx->stream, cv, ci,
                       B, G, gstride, bstride, kc, k, ov, oi, rows, nrows, dyn_items, dyn_cus);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

hnm_status hnm_topk_merge_i32(hnm_ctx* ctx, const float* cv, const int32_t* ci, int64_t B,
                              int64_t G, int64_t gstride, int64_t bstride, int kc, int k,
                              float* ov, int64_t* oi) {
  return launch_merge<int32_t>(ctx, cv, ci, B, G, gstride, bstride, kc, k, ov, oi);
}

hnm_status hnm_topk_merge_rows(hnm_ctx* ctx, const float* cv, const int32_t* ci, int64_t B,
                               int64_t G, int64_t gstride, int64_t bstride, int kc, int k,
                               float* ov, int64_t* oi, const int32_t* rows,
                               const int32_t* nrows, int64_t dyn_items, int dyn_cus) {
  return launch_merge<int32_t>(ctx, cv, ci, B, G, gstride, bstride, kc, k, ov, oi, rows, nrows,
                               dyn_items, dyn_cus);
}

// ------------------------------------------------------------------ k-th of bound lists
// One thread per row: a G-way merge of the row's G descending lists (heads and positions in
// registers, G a template constant), k pops; the k-th popped value (-inf past the union).
// The item-shard exchange's bound: ~96 values a row at G = 8, k = 12 (the wave-per-row top-K
// merge above spends ~86 us on 32k such rows; this reads each value at most once).
template <int G>
__global__ __launch_bounds__(256) void lists_kth_kernel(const float* __restrict__ L, int64_t B,
                                                        int kc, int k, float* __restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const float* row = L + b * kc;
  const int64_t gs = B * kc;
  float head[G];
  int pos[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    pos[g] = 0;
    head[g] = row[g * gs];
  }
  float v = -__builtin_inff();
  for (int r = 0; r < k; ++r) {
    int best = 0;
#pragma unroll
    for (int g = 1; g < G; ++g)
      if (head[g] > head[best]) best = g;
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (g == best) {
        v = head[g];
        ++pos[g];
        head[g] = pos[g] < kc ? row[g * gs + pos[g]] : -__builtin_inff();
      }
  }
  out[b] = v;
}

extern "C" hnm_status hnm_topk_lists_kth_f32(hnm_ctx* ctx, const float* lists, int64_t B,
                                             int64_t G, int kc, int k, float* out) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && ((lists && out) || B == 0), HNM_EINVAL, "lists_kth: NULL argument");
  HNM_REQUIRE(G >= 1 && G <= 16 && kc >= 1 && k >= 1 && k <= kc * G, HNM_EINVAL,
              "lists_kth: 1 <= G <= 16, 1 <= k <= G * kc");
  if (B <= 0) return HNM_OK;
  const dim3 grid((unsigned)hnm_cdiv(B, 256));
  switch (G) {
#define HNM_KTH(g) \
  case g: hipLaunchKernelGGL(lists_kth_kernel<g>, grid, dim3(256), 0, ctx->stream, lists, B, kc, k, out); break;
    HNM_KTH(1) HNM_KTH(2) HNM_KTH(3) HNM_KTH(4) HNM_KTH(5) HNM_KTH(6) HNM_KTH(7) HNM_KTH(8)
    HNM_KTH(9) HNM_KTH(10) HNM_KTH(11) HNM_KTH(12) HNM_KTH(13) HNM_KTH(14) HNM_KTH(15) HNM_KTH(16)
#undef HNM_KTH
  }
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

// ------------------------------------------------------------------ exchange candidates
// The item-shard exchange's candidate lists travel as int32 pairs (score bits, global item
// id): one all_to_all.  pack: shard-local ids + offset (-1 stays -1) next to the score bits.
__global__ __launch_bounds__(256) void pack_pairs_kernel(const float* __restrict__ v,
                                                         const int64_t* __restrict__ idx,
                                                         int64_t n, int64_t offset,
                                                         int2* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  const int64_t i = idx[e];
  out[e] = make_int2(__float_as_int(v[e]), i >= 0 ? (int)(i + offset) : (int)i);
}

extern "C" hnm_status hnm_pack_candidates_i32(hnm_ctx* ctx, const float* val, const int64_t* idx,
                                              int64_t n, int64_t offset, int32_t* pairs) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && ((val && idx && pairs) || n <= 0), HNM_EINVAL, "pack_candidates: NULL argument");
  HNM_REQUIRE(((uintptr_t)pairs & 7) == 0, HNM_EINVAL, "pack_candidates: pairs must be 8-byte aligned");
  if (n <= 0) return HNM_OK;
  hipLaunchKernelGGL(pack_pairs_kernel, dim3((unsigned)hnm_cdiv(n, 256)), dim3(256), 0, ctx->stream,
                     val, idx, n, offset, (int2*)pairs);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

// merge: one thread per row, a G-way merge of G lists each sorted in the top-K order (score
// desc, id asc; empty slots = id < 0 at the tail), k pops -> the same [B, k] as
// topk_merge_kernel over the same candidates (empty slots out as (-inf, -1)).
template <int G>
__global__ __launch_bounds__(256) void merge_sorted_pairs_kernel(const int2* __restrict__ P,
                                                                 int64_t B, int kc, int k,
                                                                 float* __restrict__ ov,
                                                                 int64_t* __restrict__ oi) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const int2* row = P + b * kc;
  const int64_t gs = B * kc;
  float hv[G];
  int hi[G], pos[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    pos[g] = 0;
    const int2 e = row[g * gs];
    hv[g] = e.y >= 0 ? __int_as_float(e.x) : -__builtin_inff();
    hi[g] = e.y >= 0 ? e.y : HNM_SENTINEL_IDX;
  }
  for (int r = 0; r < k; ++r) {
    int best = 0;
#pragma unroll
    for (int g = 1; g < G; ++g)
      if (hnm_better(hv[g], hi[g], hv[best], hi[best])) best = g;
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (g == best) {
        ov[b * k + r] = hv[g];
        oi[b * k + r] = hi[g] == HNM_SENTINEL_IDX ? -1 : hi[g];
        ++pos[g];
        const int2 e = pos[g] < kc ? row[g * gs + pos[g]] : make_int2(0, -1);
        hv[g] = e.y >= 0 ? __int_as_float(e.x) : -__builtin_inff();
        hi[g] = e.y >= 0 ? e.y : HNM_SENTINEL_IDX;
      }
  }
}

extern "C" hnm_status hnm_topk_merge_sorted_pairs_i32(hnm_ctx* ctx, const int32_t* pairs,
                                                      int64_t B, int64_t G, int kc, int k,
                                                      float* out_val, int64_t* out_idx) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && ((pairs && out_val && out_idx) || B == 0), HNM_EINVAL,
              "merge_sorted_pairs: NULL argument");
  HNM_REQUIRE(G >= 1 && G <= 16 && kc >= 1 && k >= 1 && k <= 128, HNM_EINVAL,
              "merge_sorted_pairs: 1 <= G <= 16, kc >= 1, 1 <= k <= 128");
  HNM_REQUIRE(((uintptr_t)pairs & 7) == 0, HNM_EINVAL, "merge_sorted_pairs: pairs must be 8-byte aligned");
  if (B <= 0) return HNM_OK;
  const dim3 grid((unsigned)hnm_cdiv(B, 256));
  const int2* P = (const int2*)pairs;
  switch (G) {
#define HNM_MSP(g) \
  case g: hipLaunchKernelGGL(merge_sorted_pairs_kernel<g>, grid, dim3(256), 0, ctx->stream, P, B, kc, k, out_val, out_idx); break;
    HNM_MSP(1) HNM_MSP(2) HNM_MSP(3) HNM_MSP(4) HNM_MSP(5) HNM_MSP(6) HNM_MSP(7) HNM_MSP(8)
    HNM_MSP(9) HNM_MSP(10) HNM_MSP(11) HNM_MSP(12) HNM_MSP(13) HNM_MSP(14) HNM_MSP(15) HNM_MSP(16)
#undef HNM_MSP
  }
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

extern "C" hnm_status hnm_topk_merge_f32(hnm_ctx* ctx, const float* cand_val,
                                         const int64_t* cand_idx, int64_t B, int64_t G,
                                         int64_t gstride, int64_t bstride, int kc, int k,
                                         float* out_val, int64_t* out_idx) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && ((cand_val && cand_idx && out_idx) || B == 0), HNM_EINVAL, "merge: NULL argument");
  HNM_REQUIRE(k >= 1 && k <= 128 && kc >= 1 && G >= 1, HNM_EINVAL, "merge: bad k/kc/G");
  if (B <= 0) return HNM_OK;
  return launch_merge<int64_t>(ctx, cand_val, cand_idx, B, G, gstride, bstride, kc, k,
                               out_val, out_idx);
}

// ------------------------------------------------------------------ pairwise dot
// out[n] = U[u[n]] . V[i[n]] (+ ub[u[n]]) (+ ib[i[n]]) (+ cb[0]); one wave per pair.
// LightGCN.predict (lightgcn.py:166-186), MatrixFactorization.forward (:80-106).
__global__ __launch_bounds__(256) void pair_dot_kernel(const float* __restrict__ U, int64_t nu,
                                                       int64_t ldu, const float* __restrict__ V,
                                                       int64_t ni, int64_t ldv, int d,
                                                       const int64_t* __restrict__ uid,
                                                       const int64_t* __restrict__ iid, int64_t n,
                                                       const float* ub, const float* ib,
                                                       const float* cb, float* __restrict__ out,
                                                       unsigned* err) {
  const int64_t e = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= n) return;
  const int lane = threadIdx.x & 63;
  const int64_t u = uid[e], i = iid[e];
  if (u < 0 || u >= nu || i < 0 || i >= ni) {
    if (lane == 0) {
      hnm_flag(err, HNM_ERR_OOB);
      out[e] = __builtin_nanf("");
    }
    return;
  }
  float acc = 0.f;
  for (int c = lane; c < d; c += 64) acc = fmaf(U[u * ldu + c], V[i * ldv + c], acc);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) {
    if (ub) acc += ub[u];
    if (ib) acc += ib[i];
    if (cb) acc += cb[0];
    out[e] = acc;
  }
}

extern "C" hnm_status hnm_pair_dot_f32(hnm_ctx* ctx, const float* user_tab, int64_t num_users,
                                       int64_t ldu, const float* item_tab, int64_t num_items,
                                       int64_t ldi, int d, const int64_t* user_ids,
                                       const int64_t* item_ids, int64_t n,
                                       const float* user_bias, const float* item_bias,
                                       const float* const_bias, float* out) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && user_tab && item_tab && ((user_ids && item_ids && out) || n == 0), HNM_EINVAL,
              "pair_dot: NULL argument");
  HNM_REQUIRE(d >= 1 && ldu >= d && ldi >= d, HNM_EINVAL, "pair_dot: bad shape");
  if (n <= 0) return HNM_OK;
  hipLaunchKernelGGL(pair_dot_kernel, dim3((unsigned)hnm_cdiv(n, 4)), dim3(256), 0, ctx->stream,
                     user_tab, num_users, ldu, item_tab, num_items, ldi, d, user_ids, item_ids, n,
                     user_bias, item_bias, const_bias, out, ctx->err_dev);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

// ------------------------------------------------------------------ a11: history mask gather
// The -inf mask of one recommend() batch from a device-resident per-user history CSR
// (the purchase-history filter of serve.py:350-352 / each recommend's filter loop,
// neural_cf.py:316-321): row b masks the ids of hist_idx[hist_ptr[u] .. hist_ptr[u + 1])
// (sorted) of u = user_ids[b] that fall in the item range [lo, hi), renumbered to i - lo
// (an item shard's local ids).  Two launches, no host sync: one workgroup scans the B row
// lengths into mask_ptr (rows of out-of-range users are empty; the scoring kernel flags
// them), then one wave per row copies its ids (coalesced int32 runs).  Offsets past
// `capacity` are clamped (the row is truncated, HNM_ERR_MASK_CAP raised) so no reader can
// run off the buffer.
__device__ __forceinline__ void hist_run(const int64_t* __restrict__ hist_ptr,
                                         const int32_t* __restrict__ hist_idx, int64_t u,
                                         int32_t lo, int32_t hi, bool whole, int64_t& a,
                                         int64_t& z) {
  a = hist_ptr[u];
  z = hist_ptr[u + 1];
  if (whole) return;
  int64_t l = a, r = z;  // first position >= lo
  while (l < r) {
    const int64_t m = (l + r) >> 1;
    if (hist_idx[m] < lo) l = m + 1;
    else r = m;
  }
  int64_t l2 = l, r2 = z;  // first position >= hi
  while (l2 < r2) {
    const int64_t m = (l2 + r2) >> 1;
    if (hist_idx[m] < hi) l2 = m + 1;
    else r2 = m;
  }
  a = l;
  z = l2;
}

__global__ __launch_bounds__(1024) void mask_scan_kernel(const int64_t* __restrict__ hist_ptr,
                                                         const int32_t* __restrict__ hist_idx,
                                                         int64_t num_users,
                                                         const int64_t* __restrict__ uid,
                                                         int64_t B, int32_t lo, int32_t hi,
                                                         bool whole, int64_t capacity,
                                                         int64_t* __restrict__ mptr,
                                                         unsigned* err) {
  __shared__ int64_t wsum[16];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t per = hnm_cdiv(B, 1024);
  const int64_t b0 = (int64_t)t * per, b1 = b0 + per < B ? b0 + per : B;
  int64_t mine = 0;
  for (int64_t b = b0; b < b1; ++b) {
    const int64_t u = uid[b];
    if (u < 0 || u >= num_users) continue;
    int64_t a, z;
    hist_run(hist_ptr, hist_idx, u, lo, hi, whole, a, z);
    mine += z - a;
  }
  // inclusive wave scan, then the 16 wave totals
  int64_t inc = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t v = __shfl_up(inc, o);
    if (lane >= o) inc += v;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  int64_t base = 0;
  for (int w = 0; w < wv; ++w) base += wsum[w];
  int64_t off = base + inc - mine;
  for (int64_t b = b0; b < b1; ++b) {
    mptr[b] = off < capacity ? off : capacity;
    const int64_t u = uid[b];
    if (u < 0 || u >= num_users) continue;
    int64_t a, z;
    hist_run(hist_ptr, hist_idx, u, lo, hi, whole, a, z);
    off += z - a;
  }
  if (t == 1023) {
    const int64_t total = base + inc;
    mptr[B] = total < capacity ? total : capacity;
    if (total > capacity) hnm_flag(err, HNM_ERR_MASK_CAP);
  }
}

__global__ __launch_bounds__(256) void mask_copy_kernel(const int64_t* __restrict__ hist_ptr,
                                                        const int32_t* __restrict__ hist_idx,
                                                        int64_t num_users,
                                                        const int64_t* __restrict__ uid, int64_t B,
                                                        int32_t lo, int32_t hi, bool whole,
                                                        const int64_t* __restrict__ mptr,
                                                        int32_t* __restrict__ midx) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  const int64_t u = uid[b];
  if (u < 0 || u >= num_users) return;
  int64_t a, z;
  hist_run(hist_ptr, hist_idx, u, lo, hi, whole, a, z);
  const int64_t dst = mptr[b], n = mptr[b + 1] - dst;
  for (int64_t j = lane; j < n; j += 64) midx[dst + j] = hist_idx[a + j] - lo;
}

extern "C" hnm_status hnm_mask_gather_csr(hnm_ctx* ctx, const int64_t* hist_ptr,
                                          const int32_t* hist_idx, int64_t num_users,
                                          const int64_t* user_ids, int64_t B, int64_t item_lo,
                                          int64_t item_hi, int64_t capacity, int64_t* mask_ptr,
                                          int32_t* mask_idx) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && hist_ptr && (user_ids || B == 0) && mask_ptr && (hist_idx || capacity == 0) &&
                  (mask_idx || capacity == 0),
              HNM_EINVAL, "mask_gather: NULL argument");
  HNM_REQUIRE(num_users >= 0 && B >= 0 && capacity >= 0 && 0 <= item_lo && item_lo <= item_hi,
              HNM_EINVAL, "mask_gather: bad size or item range");
  if (B == 0) return HNM_OK;
  const int32_t lo = (int32_t)item_lo;
  const int32_t hi = (int32_t)std::min<int64_t>(item_hi, INT32_MAX);
  const bool whole = item_lo == 0 && item_hi >= INT32_MAX;
  hipLaunchKernelGGL(mask_scan_kernel, dim3(1), dim3(1024), 0, ctx->stream, hist_ptr, hist_idx,
                     num_users, user_ids, B, lo, hi, whole, capacity, mask_ptr, ctx->err_dev);
  HNM_LAUNCH_CHECK();
  hipLaunchKernelGGL(mask_copy_kernel, dim3((unsigned)hnm_cdiv(B, 4)), dim3(256), 0, ctx->stream,
                     hist_ptr, hist_idx, num_users, user_ids, B, lo, hi, whole, mask_ptr,
                     mask_idx);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}
