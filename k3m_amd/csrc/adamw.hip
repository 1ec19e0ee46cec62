// AdamW with pytorch_transformers 1.1.0 semantics (the optimizer of train_concap_struc.py:436-441)
// over a contiguous segment of the flat parameter buffer: one launch updates every tensor of a
// weight-decay group.  HBM-bound: 16 B read + 12 B written per fp32 parameter (+2 B for the
// optional bf16 shadow used by the mixed-precision GEMMs).
#include <cmath>
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    uint16_t* __restrict__ pb, long long n4, float b1, float omb1,
                                                    float b2, float omb2, float eps, float step_size, float decay,
                                                    float gscale) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    floatx4 pp = reinterpret_cast<floatx4*>(p)[i];
    floatx4 gg = reinterpret_cast<const floatx4*>(g)[i];
    floatx4 mm = reinterpret_cast<floatx4*>(m)[i];
    floatx4 vv = reinterpret_cast<floatx4*>(v)[i];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float gr = gg[q] * gscale;
      // exp_avg.mul_(beta1).add_(1 - beta1, grad)
      mm[q] = __fadd_rn(__fmul_rn(mm[q], b1), __fmul_rn(omb1, gr));
      // exp_avg_sq.mul_(beta2).addcmul_(1 - beta2, grad, grad)
      vv[q] = __fadd_rn(__fmul_rn(vv[q], b2), __fmul_rn(__fmul_rn(omb2, gr), gr));
      // denom = exp_avg_sq.sqrt().add_(eps); p.addcdiv_(-step_size, exp_avg, denom)
      const float denom = sqrtf(vv[q]) + eps;
      pp[q] = __fadd_rn(pp[q], __fmul_rn(-step_size, __fdiv_rn(mm[q], denom)));
      // p.add_(-lr * weight_decay, p)
      if (decay != 0.f) pp[q] = __fadd_rn(pp[q], __fmul_rn(-decay, pp[q]));
    }
    reinterpret_cast<floatx4*>(p)[i] = pp;
    reinterpret_cast<floatx4*>(m)[i] = mm;
    reinterpret_cast<floatx4*>(v)[i] = vv;
    if (pb) {
      uint2 u;
      u.x = (uint32_t)from_f<bf16_t>(pp[0]).x | ((uint32_t)from_f<bf16_t>(pp[1]).x << 16);
      u.y = (uint32_t)from_f<bf16_t>(pp[2]).x | ((uint32_t)from_f<bf16_t>(pp[3]).x << 16);
      reinterpret_cast<uint2*>(pb)[i] = u;
    }
  }
}

// torch.optim.AdamW (the fine-tuning optimizer, finetune.py:356-361), foreach-path op order:
// p *= 1 - lr*wd; m = lerp(m, g, 1-b1); v = v*b2 + (1-b2) g g; p -= step_size * m / (sqrt(v)/sqrt(bc2) + eps)
__global__ __launch_bounds__(256) void adamw_torch_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                          float* __restrict__ m, float* __restrict__ v,
                                                          uint16_t* __restrict__ pb, long long n4, float omb1,
                                                          float b2, float omb2, float eps, float step_size,
                                                          float bc2_sqrt, float keep, float gscale) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    floatx4 pp = reinterpret_cast<floatx4*>(p)[i];
    floatx4 gg = reinterpret_cast<const floatx4*>(g)[i];
    floatx4 mm = reinterpret_cast<floatx4*>(m)[i];
    floatx4 vv = reinterpret_cast<floatx4*>(v)[i];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float gr = gg[q] * gscale;
      pp[q] = __fmul_rn(pp[q], keep);
      mm[q] = __fadd_rn(mm[q], __fmul_rn(omb1, __fsub_rn(gr, mm[q])));
      vv[q] = __fadd_rn(__fmul_rn(vv[q], b2), __fmul_rn(__fmul_rn(omb2, gr), gr));
      const float denom = __fadd_rn(__fdiv_rn(sqrtf(vv[q]), bc2_sqrt), eps);
      pp[q] = __fadd_rn(pp[q], __fmul_rn(-step_size, __fdiv_rn(mm[q], denom)));
    }
    reinterpret_cast<floatx4*>(p)[i] = pp;
    reinterpret_cast<floatx4*>(m)[i] = mm;
    reinterpret_cast<floatx4*>(v)[i] = vv;
    if (pb) {
      uint2 u;
      u.x = (uint32_t)from_f<bf16_t>(pp[0]).x | ((uint32_t)from_f<bf16_t>(pp[1]).x << 16);
      u.y = (uint32_t)from_f<bf16_t>(pp[2]).x | ((uint32_t)from_f<bf16_t>(pp[3]).x << 16);
      reinterpret_cast<uint2*>(pb)[i] = u;
    }
  }
}

// k3m_adamw_ex: the pytorch_transformers rule above or apex FusedAdam (adam_w_mode, the mixed-
// precision branch train_concap_struc.py:410-411, :426): m, v as above;
//   p -= lr * ((m / bc1) / (sqrt(v / bc2) + eps) + wd * p)      (bc = 1 without bias correction)
// flags & K3M_ADAM_ZERO_GRAD: g is zeroed after it is read (optimizer.zero_grad() fused: the
// gradient buffer is not swept a second time).
template <bool APEX, bool ZERO>
__global__ __launch_bounds__(256) void adamw_ex_kernel(float* __restrict__ p, float* __restrict__ g,
                                                       float* __restrict__ m, float* __restrict__ v,
                                                       uint16_t* __restrict__ pb, long long n4, float b1, float omb1,
                                                       float b2, float omb2, float eps, float step_size, float decay,
                                                       float gscale, float rbc1, float rbc2,
                                                       const float* __restrict__ sc) {
  if (sc) {   // k3m_adamw_ex_dev: the step's scalars from device memory (a hipGraph-captured launch)
    step_size = sc[0];
    decay = sc[1];
    rbc1 = sc[2];
    rbc2 = sc[3];
  }
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    floatx4 pp = reinterpret_cast<floatx4*>(p)[i];
    floatx4 gg = reinterpret_cast<const floatx4*>(g)[i];
    floatx4 mm = reinterpret_cast<floatx4*>(m)[i];
    floatx4 vv = reinterpret_cast<floatx4*>(v)[i];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float gr = gg[q] * gscale;
      mm[q] = __fadd_rn(__fmul_rn(mm[q], b1), __fmul_rn(omb1, gr));
      vv[q] = __fadd_rn(__fmul_rn(vv[q], b2), __fmul_rn(__fmul_rn(omb2, gr), gr));
      if constexpr (APEX) {
        const float denom = __fadd_rn(sqrtf(__fmul_rn(vv[q], rbc2)), eps);
        const float upd = __fadd_rn(__fdiv_rn(__fmul_rn(mm[q], rbc1), denom), __fmul_rn(decay, pp[q]));
        pp[q] = __fsub_rn(pp[q], __fmul_rn(step_size, upd));
      } else {
        const float denom = sqrtf(vv[q]) + eps;
        pp[q] = __fadd_rn(pp[q], __fmul_rn(-step_size, __fdiv_rn(mm[q], denom)));
        if (decay != 0.f) pp[q] = __fadd_rn(pp[q], __fmul_rn(-decay, pp[q]));
      }
    }
    reinterpret_cast<floatx4*>(p)[i] = pp;
    reinterpret_cast<floatx4*>(m)[i] = mm;
    reinterpret_cast<floatx4*>(v)[i] = vv;
    if constexpr (ZERO) reinterpret_cast<floatx4*>(g)[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (pb) {
      uint2 u;
      u.x = (uint32_t)from_f<bf16_t>(pp[0]).x | ((uint32_t)from_f<bf16_t>(pp[1]).x << 16);
      u.y = (uint32_t)from_f<bf16_t>(pp[2]).x | ((uint32_t)from_f<bf16_t>(pp[3]).x << 16);
      reinterpret_cast<uint2*>(pb)[i] = u;
    }
  }
}

}  // namespace

// (step_size, decay, 1/bc1, 1/bc2) of one k3m_adamw_ex launch, in double on the host, rounded once
static void adam_scalars(double lr, double beta1, double beta2, double wd, int step, int flags, float* out) {
  float step_size, decay, rbc1 = 1.f, rbc2 = 1.f;
  if (flags & K3M_ADAM_APEX) {
    if (flags & K3M_ADAM_APEX_BIAS_CORRECTION) {
      rbc1 = (float)(1.0 / (1.0 - std::pow(beta1, step)));
      rbc2 = (float)(1.0 / (1.0 - std::pow(beta2, step)));
    }
    step_size = (float)lr;
    decay = (float)wd;
  } else {
    const double bc1 = 1.0 - std::pow(beta1, step), bc2 = 1.0 - std::pow(beta2, step);
    step_size = (float)(lr * std::sqrt(bc2) / bc1);
    decay = wd > 0.0 ? (float)(lr * wd) : 0.f;
  }
  out[0] = step_size;
  out[1] = decay;
  out[2] = rbc1;
  out[3] = rbc2;
}

static int adamw_ex_launch(float* p, float* g, float* m, float* v, uint16_t* p_bf16, long long n, const float* s4,
                           const float* dev_sc, double beta1, double beta2, double eps, float grad_scale, int flags,
                           hipStream_t st) {
  K3M_ARG(p && g && m && v && n >= 0 && n % 4 == 0);
  K3M_ARG(((uintptr_t)p & 15) == 0 && ((uintptr_t)g & 15) == 0 && ((uintptr_t)m & 15) == 0 && ((uintptr_t)v & 15) == 0);
  K3M_ARG((flags & ~(K3M_ADAM_ZERO_GRAD | K3M_ADAM_APEX | K3M_ADAM_APEX_BIAS_CORRECTION)) == 0);
  if (n == 0) return 0;
  const long long n4 = n / 4;
  const int blocks = (int)std::min<long long>((n4 + 255) / 256, 256 * 16);
  const bool apex = (flags & K3M_ADAM_APEX) != 0, zero = (flags & K3M_ADAM_ZERO_GRAD) != 0;
#define K3M_ADAM_LAUNCH(A, Z)                                                                                      \
  hipLaunchKernelGGL((adamw_ex_kernel<A, Z>), dim3(blocks), dim3(256), 0, st, p, g, m, v, p_bf16, n4, (float)beta1, \
                     (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps, s4[0], s4[1], grad_scale,  \
                     s4[2], s4[3], dev_sc)
  if (apex) {
    if (zero) K3M_ADAM_LAUNCH(true, true);
    else K3M_ADAM_LAUNCH(true, false);
  } else {
    if (zero) K3M_ADAM_LAUNCH(false, true);
    else K3M_ADAM_LAUNCH(false, false);
  }
#undef K3M_ADAM_LAUNCH
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_adamw_ex(float* p, float* g, float* m, float* v, uint16_t* p_bf16, long long n, double lr,
                            double beta1, double beta2, double eps, double wd, int step, float grad_scale, int flags,
                            hipStream_t st) {
  K3M_ARG(step >= 1);
  float s4[4];
  adam_scalars(lr, beta1, beta2, wd, step, flags, s4);
  return adamw_ex_launch(p, g, m, v, p_bf16, n, s4, nullptr, beta1, beta2, eps, grad_scale, flags, st);
}

extern "C" int k3m_adamw_ex_dev(float* p, float* g, float* m, float* v, uint16_t* p_bf16, long long n,
                                const float* scalars, double beta1, double beta2, double eps, float grad_scale,
                                int flags, hipStream_t st) {
  K3M_ARG(scalars && ((uintptr_t)scalars & 15) == 0);
  const float zero4[4] = {0.f, 0.f, 0.f, 0.f};
  return adamw_ex_launch(p, g, m, v, p_bf16, n, zero4, scalars, beta1, beta2, eps, grad_scale, flags, st);
}

extern "C" int k3m_adamw_scalars_n(int n, const double* lr, const double* wd, double beta1, double beta2, int step,
                                   int flags, float* out) {
  K3M_ARG(n >= 0 && (n == 0 || (lr && wd && out)) && step >= 1);
  K3M_ARG((flags & ~(K3M_ADAM_ZERO_GRAD | K3M_ADAM_APEX | K3M_ADAM_APEX_BIAS_CORRECTION)) == 0);
  for (int i = 0; i < n; ++i) adam_scalars(lr[i], beta1, beta2, wd[i], step, flags, out + 4 * i);
  return 0;
}

extern "C" int k3m_adamw_torch(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, long long n, double lr,
                               double beta1, double beta2, double eps, double wd, int step, float grad_scale,
                               hipStream_t st) {
  K3M_ARG(p && g && m && v && n >= 0 && n % 4 == 0 && step >= 1);
  K3M_ARG(((uintptr_t)p & 15) == 0 && ((uintptr_t)g & 15) == 0 && ((uintptr_t)m & 15) == 0 && ((uintptr_t)v & 15) == 0);
  if (n == 0) return 0;
  const double bc1 = 1.0 - std::pow(beta1, step), bc2 = 1.0 - std::pow(beta2, step);
  const long long n4 = n / 4;
  const int blocks = (int)std::min<long long>((n4 + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(adamw_torch_kernel, dim3(blocks), dim3(256), 0, st, p, g, m, v, p_bf16, n4, (float)(1.0 - beta1),
                     (float)beta2, (float)(1.0 - beta2), (float)eps, (float)(lr / bc1), (float)std::sqrt(bc2),
                     (float)(1.0 - lr * wd), grad_scale);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_adamw(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, long long n, double lr,
                         double beta1, double beta2, double eps, double wd, int step, float grad_scale, hipStream_t st) {
  K3M_ARG(p && g && m && v && n >= 0 && n % 4 == 0 && step >= 1);
  K3M_ARG(((uintptr_t)p & 15) == 0 && ((uintptr_t)g & 15) == 0 && ((uintptr_t)m & 15) == 0 && ((uintptr_t)v & 15) == 0);
  if (n == 0) return 0;
  const double bc1 = 1.0 - std::pow(beta1, step), bc2 = 1.0 - std::pow(beta2, step);
  const float step_size = (float)(lr * std::sqrt(bc2) / bc1);
  const float decay = wd > 0.0 ? (float)(lr * wd) : 0.f;
  const long long n4 = n / 4;
  const int blocks = (int)std::min<long long>((n4 + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(adamw_kernel, dim3(blocks), dim3(256), 0, st, p, g, m, v, p_bf16, n4, (float)beta1,
                     (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps, step_size, decay, grad_scale);
  K3M_CHECK_LAUNCH();
  return 0;
}
