// PyTorch operator registrations for the gfx950 HIP kernels.
//
// Ops live in the `bpe_hip` namespace (torch.ops.bpe_hip.*) and are registered
// for the CUDA dispatch key, which is what ROCm PyTorch uses for HIP device
// tensors.  Each op validates shapes/dtypes on the host (so no kernel ever
// sees a shape it was not written for), allocates outputs through the caching
// allocator and launches on the current HIP stream -- no syncs, so the ops are
// safe inside HIP-graph capture.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "kernels.h"

#include <algorithm>

namespace {

// ROCm PyTorch exposes HIP devices under the CUDA device type ("masquerading"),
// so guards and streams must come from the masquerading variants.
hipStream_t cur_stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }
using DevGuard = at::hip::HIPGuardMasqueradingAsCUDA;

int dt_code(const at::Tensor& t) {
    if (t.scalar_type() == at::kBFloat16) return DT_BF16;
    if (t.scalar_type() == at::kFloat) return DT_F32;
    TORCH_CHECK(false, "bpe_hip: only float32 / bfloat16 tensors are supported, got ", t.scalar_type());
    return -1;
}
int vec_elems(const at::Tensor& t) { return dt_code(t) == DT_BF16 ? 8 : 4; }

void check_cuda(const at::Tensor& t, const char* name) {
    TORCH_CHECK(t.is_cuda(), "bpe_hip: ", name, " must be a GPU tensor");
}
void check_aligned(const at::Tensor& t, const char* name) {
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "bpe_hip: ", name,
                " must be 16-byte aligned");
}

// ---------------------------------------------------------------- RMSNorm
// s = x + d (stored), y = RMSNorm(s) -> (s, y, rstd)
std::tuple<at::Tensor, at::Tensor, at::Tensor> add_rmsnorm_fwd(const at::Tensor& x, const at::Tensor& d,
                                                               const at::Tensor& w, double eps) {
    check_cuda(x, "x");
    TORCH_CHECK(x.is_contiguous() && d.is_contiguous() && w.is_contiguous(), "add_rmsnorm: contiguous inputs required");
    TORCH_CHECK(x.scalar_type() == w.scalar_type() && d.scalar_type() == x.scalar_type(), "add_rmsnorm: dtypes differ");
    TORCH_CHECK(d.sizes() == x.sizes(), "add_rmsnorm: x and d shapes differ");
    const int N = (int)x.size(-1);
    TORCH_CHECK(w.numel() == N, "add_rmsnorm: weight size mismatch");
    TORCH_CHECK(N % vec_elems(x) == 0, "add_rmsnorm: last dim must be a multiple of 8 (bf16) / 4 (fp32)");
    check_aligned(x, "x");
    check_aligned(d, "d");
    const int M = (int)(x.numel() / N);
    DevGuard g(x.device());
    auto sum = at::empty_like(x);
    auto y = at::empty_like(x);
    auto rstd = at::empty({M}, x.options().dtype(at::kFloat));
    launch_add_rmsnorm_fwd(dt_code(x), x.data_ptr(), d.data_ptr(), w.data_ptr(), sum.data_ptr(), y.data_ptr(),
                           rstd.data_ptr<float>(), M, N, (float)eps, cur_stream());
    return {sum, y, rstd};
}

std::tuple<at::Tensor, at::Tensor> rmsnorm_fwd(const at::Tensor& x, const at::Tensor& w, double eps) {
    check_cuda(x, "x");
    TORCH_CHECK(x.is_contiguous() && w.is_contiguous(), "rmsnorm: contiguous inputs required");
    TORCH_CHECK(x.scalar_type() == w.scalar_type(), "rmsnorm: x and weight dtypes differ");
    const int N = (int)x.size(-1);
    TORCH_CHECK(w.numel() == N, "rmsnorm: weight size mismatch");
    TORCH_CHECK(N % vec_elems(x) == 0, "rmsnorm: last dim must be a multiple of 8 (bf16) / 4 (fp32)");
    check_aligned(x, "x");
    const int M = (int)(x.numel() / N);
    DevGuard g(x.device());
    auto y = at::empty_like(x);
    auto rstd = at::empty({M}, x.options().dtype(at::kFloat));
    launch_rmsnorm_fwd(dt_code(x), x.data_ptr(), w.data_ptr(), y.data_ptr(), rstd.data_ptr<float>(), M, N, (float)eps,
                       cur_stream());
    return {y, rstd};
}

// dw_acc: add dw into this (bf16 or fp32, contiguous, N elements: a parameter's flat gradient slot) instead of
// returning it (the second output is then empty)
std::tuple<at::Tensor, at::Tensor> rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                                               const at::Tensor& rstd, const c10::optional<at::Tensor>& dres,
                                               const c10::optional<at::Tensor>& dw_acc) {
    check_cuda(x, "x");
    auto dyc = dy.contiguous();
    const int N = (int)x.size(-1);
    const int M = (int)(x.numel() / N);
    const int nv = N / vec_elems(x);
    TORCH_CHECK(N <= 8 * 64 * vec_elems(x) || (N % vec_elems(x) == 0 && nv % 256 == 0 && nv <= 1024),
                "rmsnorm bwd: hidden size too large");
    TORCH_CHECK(dyc.scalar_type() == x.scalar_type(), "rmsnorm bwd: dtype mismatch");
    DevGuard g(x.device());
    auto dx = at::empty_like(x);
    const bool acc = dw_acc.has_value() && dw_acc->defined();
    int mode = 0;
    if (acc) {
        TORCH_CHECK(dw_acc->is_contiguous() && dw_acc->numel() == N && dw_acc->device() == x.device() &&
                        (dw_acc->scalar_type() == at::kBFloat16 || dw_acc->scalar_type() == at::kFloat),
                    "rmsnorm bwd: dw_acc must be a contiguous bf16 / fp32 [N] tensor on the device");
        mode = dw_acc->scalar_type() == at::kFloat ? 2 : 1;
    }
    auto dw = acc ? at::empty({0}, w.options()) : at::empty_like(w);
    const int grid = rmsnorm_bwd_grid(M);
    auto partial = at::empty({grid, N}, x.options().dtype(at::kFloat));
    const void* rp = nullptr;
    at::Tensor rc;
    if (dres.has_value() && dres->defined()) {
        rc = dres->contiguous();
        TORCH_CHECK(rc.numel() == x.numel() && rc.scalar_type() == x.scalar_type(), "rmsnorm bwd: bad residual grad");
        rp = rc.data_ptr();
    }
    launch_rmsnorm_bwd(dt_code(x), dyc.data_ptr(), x.data_ptr(), w.data_ptr(), rstd.data_ptr<float>(), dx.data_ptr(),
                       partial.data_ptr<float>(), acc ? dw_acc->data_ptr() : dw.data_ptr(), rp, M, N, cur_stream(),
                       mode);
    return {dx, dw};
}

// ---------------------------------------------------------------- activations
at::Tensor swiglu_fwd(const at::Tensor& gu) {
    check_cuda(gu, "gu");
    TORCH_CHECK(gu.is_contiguous(), "swiglu: contiguous input required");
    const int64_t F2 = gu.size(-1);
    TORCH_CHECK(F2 % (2 * vec_elems(gu)) == 0, "swiglu: hidden size must be a multiple of 8/16");
    const int F = (int)(F2 / 2);
    const size_t M = gu.numel() / F2;
    auto sizes = gu.sizes().vec();
    sizes.back() = F;
    DevGuard g(gu.device());
    auto out = at::empty(sizes, gu.options());
    launch_swiglu_fwd(dt_code(gu), gu.data_ptr(), out.data_ptr(), M, F, cur_stream());
    return out;
}

at::Tensor swiglu_bwd(const at::Tensor& dout, const at::Tensor& gu) {
    check_cuda(gu, "gu");
    auto d = dout.contiguous();
    const int64_t F2 = gu.size(-1);
    const int F = (int)(F2 / 2);
    const size_t M = gu.numel() / F2;
    DevGuard g(gu.device());
    auto dgu = at::empty_like(gu);
    launch_swiglu_bwd(dt_code(gu), d.data_ptr(), gu.data_ptr(), dgu.data_ptr(), M, F, cur_stream());
    return dgu;
}

at::Tensor act_fwd(const at::Tensor& x, int64_t kind) {
    check_cuda(x, "x");
    TORCH_CHECK(x.is_contiguous() && x.numel() % vec_elems(x) == 0, "act: contiguous, numel multiple of 8/4");
    DevGuard g(x.device());
    auto y = at::empty_like(x);
    launch_act_fwd(dt_code(x), (int)kind, x.data_ptr(), y.data_ptr(), x.numel(), cur_stream());
    return y;
}

at::Tensor act_bwd(const at::Tensor& dy, const at::Tensor& x, int64_t kind) {
    check_cuda(x, "x");
    auto d = dy.contiguous();
    DevGuard g(x.device());
    auto dx = at::empty_like(x);
    launch_act_bwd(dt_code(x), (int)kind, d.data_ptr(), x.data_ptr(), dx.data_ptr(), x.numel(), cur_stream());
    return dx;
}

// ---------------------------------------------------------------- cross entropy
// nvalid (optional fp32 scalar): the gradient's 1 / n denominator when this call covers only a slice of the
// rows (chunked LM head); default = the valid targets of this call
std::tuple<at::Tensor, at::Tensor> ce_fwd_bwd(at::Tensor logits, const at::Tensor& targets, int64_t ignore_index,
                                              bool write_grad, const c10::optional<at::Tensor>& nvalid_in) {
    check_cuda(logits, "logits");
    TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "ce: logits must be [M, V] with unit column stride");
    TORCH_CHECK(targets.scalar_type() == at::kLong && targets.is_contiguous(), "ce: targets must be int64");
    const int M = (int)logits.size(0), V = (int)logits.size(1);
    TORCH_CHECK(targets.numel() == M, "ce: targets size mismatch");
    DevGuard g(logits.device());
    auto loss = at::empty({M}, logits.options().dtype(at::kFloat));
    auto lse = at::empty({M}, logits.options().dtype(at::kFloat));
    at::Tensor nvalid;
    if (nvalid_in.has_value() && nvalid_in->defined()) {
        TORCH_CHECK(nvalid_in->scalar_type() == at::kFloat && nvalid_in->numel() == 1 && nvalid_in->is_cuda(),
                    "ce: nvalid must be a fp32 scalar on the device");
        nvalid = *nvalid_in;
    } else {
        nvalid = targets.ne(ignore_index).sum().to(at::kFloat);
    }
    launch_ce_fwd_bwd(dt_code(logits), logits.data_ptr(), logits.stride(0), targets.data_ptr<int64_t>(),
                      loss.data_ptr<float>(), lse.data_ptr<float>(), nvalid.data_ptr<float>(), M, V, ignore_index,
                      write_grad ? 1 : 0, cur_stream());
    return {loss, lse};
}

// ---------------------------------------------------------------- embedding
at::Tensor embed_fwd(const at::Tensor& W, const at::Tensor& ids) {
    check_cuda(W, "weight");
    TORCH_CHECK(W.dim() == 2 && W.is_contiguous(), "embed: weight must be contiguous [V, D]");
    TORCH_CHECK(ids.scalar_type() == at::kLong, "embed: ids must be int64");
    const int D = (int)W.size(1);
    TORCH_CHECK(D % vec_elems(W) == 0 && (D * W.element_size()) % 16 == 0, "embed: D must be a multiple of 16 bytes");
    auto idc = ids.contiguous();
    const int M = (int)idc.numel();
    auto sizes = idc.sizes().vec();
    sizes.push_back(D);
    DevGuard g(W.device());
    auto out = at::empty(sizes, W.options());
    launch_embed_fwd(dt_code(W), W.data_ptr(), idc.data_ptr<int64_t>(), out.data_ptr(), M, D, W.size(0), cur_stream());
    return out;
}

at::Tensor embed_bwd(const at::Tensor& dout, const at::Tensor& ids, int64_t vocab) {
    check_cuda(dout, "dout");
    const int D = (int)dout.size(-1);
    TORCH_CHECK(D <= 16 * 64 * vec_elems(dout), "embed bwd: D too large");
    auto d = dout.contiguous().view({-1, D});
    auto flat = ids.contiguous().view({-1});
    DevGuard g(dout.device());
    auto sorted = at::sort(flat, /*stable=*/true, /*dim=*/0, /*descending=*/false);
    auto dW = at::zeros({vocab, D}, dout.options());
    launch_embed_bwd(dt_code(dout), d.data_ptr(), std::get<0>(sorted).data_ptr<int64_t>(),
                     std::get<1>(sorted).data_ptr<int64_t>(), dW.data_ptr(), (int)flat.numel(), D, cur_stream());
    return dW;
}

// ---------------------------------------------------------------- optimizer
void adamw_step(at::Tensor p, at::Tensor m, at::Tensor v, const at::Tensor& grad, const c10::optional<at::Tensor>& pout,
                double lr, double b1, double b2, double eps, double wd, double bc1, double bc2_sqrt,
                const c10::optional<at::Tensor>& gscale, const c10::optional<at::Tensor>& nstep,
                const c10::optional<at::Tensor>& wd_mask) {
    check_cuda(p, "param");
    TORCH_CHECK(p.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat,
                "adamw: master param / moments must be fp32");
    TORCH_CHECK(p.is_contiguous() && m.is_contiguous() && v.is_contiguous() && grad.is_contiguous(),
                "adamw: contiguous buffers required");
    TORCH_CHECK(p.numel() == grad.numel() && p.numel() == m.numel() && p.numel() == v.numel(), "adamw: size mismatch");
    void* po = nullptr;
    if (pout.has_value() && pout->defined()) {
        TORCH_CHECK(pout->scalar_type() == at::kBFloat16 && pout->numel() == p.numel() && pout->is_contiguous(),
                    "adamw: param copy-out must be contiguous bf16");
        po = pout->data_ptr();
    }
    const float* gs = nullptr;
    if (gscale.has_value() && gscale->defined()) gs = gscale->data_ptr<float>();
    const int* ns = nullptr;
    if (nstep.has_value() && nstep->defined()) {
        TORCH_CHECK(nstep->scalar_type() == at::kInt && nstep->numel() == 1 && nstep->device() == p.device(),
                    "adamw: nstep must be a one-element int32 tensor on the parameters' device");
        ns = nstep->data_ptr<int>();
    }
    const uint8_t* wm = nullptr;  // one byte per 64 elements: weight decay applies where nonzero
    if (wd_mask.has_value() && wd_mask->defined()) {
        TORCH_CHECK(wd_mask->scalar_type() == at::kByte && wd_mask->is_contiguous() &&
                        wd_mask->device() == p.device() && wd_mask->numel() >= (p.numel() + 63) / 64,
                    "adamw: wd_mask must be a contiguous uint8 tensor of one byte per 64 elements");
        wm = wd_mask->data_ptr<uint8_t>();
    }
    DevGuard g(p.device());
    launch_adamw(dt_code(grad), p.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), grad.data_ptr(), po,
                 p.numel(), (float)lr, b1, b2, (float)eps, (float)wd, (float)bc1, (float)bc2_sqrt, gs, ns, wm,
                 cur_stream());
}

void adam_count_step(at::Tensor nstep, const c10::optional<at::Tensor>& gscale) {
    check_cuda(nstep, "nstep");
    TORCH_CHECK(nstep.scalar_type() == at::kInt && nstep.numel() == 1, "adam_count_step: one-element int32 tensor");
    const float* gs = nullptr;
    if (gscale.has_value() && gscale->defined()) gs = gscale->data_ptr<float>();
    DevGuard g(nstep.device());
    launch_adam_count(nstep.data_ptr<int>(), gs, cur_stream());
}

std::tuple<at::Tensor, at::Tensor> grad_norm(at::TensorList tensors, double max_norm) {
    TORCH_CHECK(!tensors.empty(), "grad_norm: empty list");
    DevGuard g(tensors[0].device());
    constexpr int NB = 2048;  // 8 blocks per CU: 256 ran the 324 MB GPT-2 gradient at 2.3 TB/s
    auto partial = at::zeros({(int64_t)tensors.size() * NB}, tensors[0].options().dtype(at::kFloat));
    for (size_t i = 0; i < tensors.size(); ++i) {
        auto t = tensors[i];
        TORCH_CHECK(t.is_contiguous(), "grad_norm: contiguous tensors required");
        check_aligned(t, "grad");
        launch_sumsq_partial(dt_code(t), t.data_ptr(), t.numel(), partial.data_ptr<float>() + i * NB, NB,
                             cur_stream());
    }
    auto norm = at::empty({}, partial.options());
    auto coef = at::empty({}, partial.options());
    launch_norm_finalize(partial.data_ptr<float>(), (int)partial.numel(), (float)max_norm, norm.data_ptr<float>(),
                         coef.data_ptr<float>(), cur_stream());
    return {norm, coef};
}

void scale_(at::Tensor x, const at::Tensor& coef) {
    check_cuda(x, "x");
    TORCH_CHECK(x.is_contiguous(), "scale_: contiguous tensor required");
    check_aligned(x, "x");
    DevGuard g(x.device());
    launch_scale(dt_code(x), x.data_ptr(), x.numel(), coef.data_ptr<float>(), cur_stream());
}

// ---------------------------------------------------------------- generic masked SDPA (contract K7)
// q [BH, Sq, D], k [BH, Sk, D], v [BH, Sk, Dv] (fp32 or bf16, one dtype); mask: bool / uint8 viewable as
// [BH, Sq, Sk] with any strides (0 for broadcast dims), or None.  fp32 math; returns [BH, Sq, Dv] in q's dtype.
at::Tensor masked_sdpa(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                       const c10::optional<at::Tensor>& mask, double scale) {
    check_cuda(q, "q");
    TORCH_CHECK(q.dim() == 3 && k.dim() == 3 && v.dim() == 3, "masked_sdpa: q / k / v must be [BH, S, D]");
    TORCH_CHECK(k.scalar_type() == q.scalar_type() && v.scalar_type() == q.scalar_type(),
                "masked_sdpa: q, k, v must share a dtype");
    const int64_t BH = q.size(0), Sq = q.size(1), D = q.size(2), Sk = k.size(1), Dv = v.size(2);
    TORCH_CHECK(k.size(0) == BH && v.size(0) == BH && k.size(2) == D && v.size(1) == Sk,
                "masked_sdpa: shape mismatch");
    TORCH_CHECK(D >= 1 && D <= 128 && Dv >= 1 && Dv <= 128, "masked_sdpa: head dims must be 1..128");
    TORCH_CHECK(BH <= 65535 && Sk >= 1, "masked_sdpa: at most 65535 batch-heads, at least one key");
    auto qc = q.contiguous(), kc = k.contiguous(), vc = v.contiguous();
    const uint8_t* mp = nullptr;
    long msb = 0, msq = 0, msk = 0;
    at::Tensor m;
    if (mask.has_value() && mask->defined()) {
        m = *mask;
        TORCH_CHECK(m.dim() == 3 && m.size(0) == BH && m.size(1) == Sq && m.size(2) == Sk,
                    "masked_sdpa: mask must be viewable as [BH, Sq, Sk]");
        TORCH_CHECK(m.is_cuda() && m.device() == q.device(), "masked_sdpa: mask must be on q's device");
        if (m.scalar_type() != at::kBool && m.scalar_type() != at::kByte) m = m.ne(0);
        mp = reinterpret_cast<const uint8_t*>(m.data_ptr());
        msb = m.stride(0);
        msq = m.stride(1);
        msk = m.stride(2);
    }
    DevGuard g(q.device());
    auto o = at::empty({BH, Sq, Dv}, q.options());
    launch_masked_sdpa(dt_code(qc), qc.data_ptr(), kc.data_ptr(), vc.data_ptr(), mp, msb, msq, msk, o.data_ptr(),
                       (int)BH, (int)Sq, (int)Sk, (int)D, (int)Dv, (float)scale, cur_stream());
    return o;
}

// ---------------------------------------------------------------- softmax
at::Tensor softmax_fwd(const at::Tensor& x) {
    check_cuda(x, "x");
    auto xc = x.contiguous();
    const int N = (int)xc.size(-1);
    const int M = (int)(xc.numel() / std::max(N, 1));
    DevGuard g(x.device());
    auto y = at::empty_like(xc);
    launch_softmax_fwd(dt_code(xc), xc.data_ptr(), y.data_ptr(), M, N, cur_stream());
    return y;
}

at::Tensor softmax_bwd(const at::Tensor& dy, const at::Tensor& y) {
    check_cuda(y, "y");
    auto d = dy.contiguous();
    const int N = (int)y.size(-1);
    const int M = (int)(y.numel() / std::max(N, 1));
    DevGuard g(y.device());
    auto dx = at::empty_like(y);
    launch_softmax_bwd(dt_code(y), d.data_ptr(), y.data_ptr(), dx.data_ptr(), M, N, cur_stream());
    return dx;
}

// ---------------------------------------------------------------- GEMM (split-K, transposed-LDS operands)
// C[Mo, No] = beta * C + op(A) . op(B); A is [Mo, R] (a_kmajor) or [R, Mo]; B is [No, R] (b_kmajor) or [R, No].
void gemm(const at::Tensor& A, bool a_kmajor, const at::Tensor& B, bool b_kmajor, at::Tensor C, double beta,
          int64_t splits, int64_t tile) {
    check_cuda(C, "C");
    TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16 &&
                    (C.scalar_type() == at::kBFloat16 || C.scalar_type() == at::kFloat),
                "gemm: bf16 operands and a bf16 or fp32 output required");
    const bool c32 = C.scalar_type() == at::kFloat;
    TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2 && A.stride(1) == 1 && B.stride(1) == 1 &&
                    C.stride(1) == 1, "gemm: 2-D row-major operands required");
    const int Mo = (int)C.size(0), No = (int)C.size(1);
    const int R = (int)(a_kmajor ? A.size(1) : A.size(0));
    TORCH_CHECK((a_kmajor ? A.size(0) : A.size(1)) == Mo, "gemm: A / C shape mismatch");
    TORCH_CHECK((b_kmajor ? B.size(0) : B.size(1)) == No && (b_kmajor ? B.size(1) : B.size(0)) == R,
                "gemm: B shape mismatch");
    TORCH_CHECK(tile == 128 || (tile == 256 && !a_kmajor && !b_kmajor),
                "gemm: tile must be 128, or 256 with both operands token-major (weight-gradient layout)");
    TORCH_CHECK(gemm_shape_ok(Mo, No, R, (int)splits, (int)tile),
                "gemm: Mo/No must be multiples of the tile and R of 64*splits");
    TORCH_CHECK(A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0 && C.stride(0) % 4 == 0, "gemm: 16-byte row alignment");
    DevGuard g(C.device());
    at::Tensor slab;
    if (splits > 1 || c32) slab = at::empty({splits, Mo, No}, C.options().dtype(at::kFloat));
    launch_gemm(a_kmajor, b_kmajor, A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), C.data_ptr(), C.stride(0),
                (float)beta, Mo, No, R, (int)splits, slab.defined() ? slab.data_ptr<float>() : nullptr, (int)tile,
                c32 ? 1 : 0, cur_stream());
}

// 8-wave ping-pong GEMM (256 x 256 x 64 tiles): same operand convention as gemm(); any layout pair.
void gemm_pp(const at::Tensor& A, bool a_kmajor, const at::Tensor& B, bool b_kmajor, at::Tensor C, double beta,
             int64_t splits) {
    check_cuda(C, "C");
    TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16 &&
                    (C.scalar_type() == at::kBFloat16 || C.scalar_type() == at::kFloat),
                "gemm_pp: bf16 operands and a bf16 or fp32 output required");
    const bool c32 = C.scalar_type() == at::kFloat;
    TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2 && A.stride(1) == 1 && B.stride(1) == 1 &&
                    C.stride(1) == 1, "gemm_pp: 2-D row-major operands required");
    TORCH_CHECK(A.device() == C.device() && B.device() == C.device(), "gemm_pp: operands on different devices");
    const int M = (int)C.size(0), N = (int)C.size(1);
    const int R = (int)(a_kmajor ? A.size(1) : A.size(0));
    TORCH_CHECK((a_kmajor ? A.size(0) : A.size(1)) == M, "gemm_pp: A / C shape mismatch");
    TORCH_CHECK((b_kmajor ? B.size(0) : B.size(1)) == N && (b_kmajor ? B.size(1) : B.size(0)) == R,
                "gemm_pp: B shape mismatch");
    TORCH_CHECK(gemm_pp_shape_ok(M, N, R, (int)splits), "gemm_pp: M, N must be multiples of 256, R of 64 (>= splits)");
    TORCH_CHECK(A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0 && C.stride(0) % 8 == 0, "gemm_pp: 16-byte row alignment");
    TORCH_CHECK((A.stride(0) * 256) < (1L << 31) && (B.stride(0) * 256) < (1L << 31),
                "gemm_pp: leading dimension too large for 32-bit tile offsets");
    DevGuard g(C.device());
    at::Tensor slab;
    if (splits > 1 || c32) slab = at::empty({splits, M, N}, C.options().dtype(at::kFloat));
    launch_gemm_pp(a_kmajor, b_kmajor, A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), C.data_ptr(),
                   C.stride(0), (float)beta, M, N, R, (int)splits, slab.defined() ? slab.data_ptr<float>() : nullptr,
                   c32 ? 1 : 0, cur_stream());
}

// Grouped weight gradients (gemm_pp.hip gemm_pp_dw_group): gs[p] = beta * gs[p] + dys[p]^T xs[p] for up to 4
// problems over the same R tokens in ONE split-K launch plus one ordered reduce.  dys[p] [R, M_p] token-major;
// xs[p] [R, N_p] token-major, or X^T [N_p, R] with x_kmajor; gs[p] [M_p, N_p], all bf16 or all fp32.
void gemm_pp_dw_group(at::TensorList gs, at::TensorList dys, at::TensorList xs, bool x_kmajor, int64_t splits,
                      double beta) {
    const int np = (int)gs.size();
    TORCH_CHECK(np >= 1 && np <= 4 && (int)dys.size() == np && (int)xs.size() == np,
                "gemm_pp_dw_group: 1-4 problems, one dY and one X per gradient");
    const bool c32 = gs[0].scalar_type() == at::kFloat;
    const void* A[4];
    const void* B[4];
    void* C[4];
    long lda[4], ldb[4], ldc[4];
    int M[4], N[4];
    const int R = (int)dys[0].size(0);
    long slab_elems = 0;
    for (int p = 0; p < np; ++p) {
        const at::Tensor& g = gs[p];
        const at::Tensor& dy = dys[p];
        const at::Tensor& x = xs[p];
        check_cuda(g, "g");
        TORCH_CHECK(g.scalar_type() == gs[0].scalar_type() &&
                        (g.scalar_type() == at::kBFloat16 || g.scalar_type() == at::kFloat) &&
                        dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16,
                    "gemm_pp_dw_group: bf16 operands, gradients all bf16 or all fp32");
        TORCH_CHECK(g.dim() == 2 && dy.dim() == 2 && x.dim() == 2 && g.stride(1) == 1 && dy.stride(1) == 1 &&
                        x.stride(1) == 1, "gemm_pp_dw_group: 2-D row-major operands required");
        TORCH_CHECK(dy.device() == g.device() && x.device() == g.device() && g.device() == gs[0].device(),
                    "gemm_pp_dw_group: operands on different devices");
        M[p] = (int)g.size(0);
        N[p] = (int)g.size(1);
        TORCH_CHECK(dy.size(0) == R && dy.size(1) == M[p], "gemm_pp_dw_group: dY [R, M] with one R for all problems");
        TORCH_CHECK(x_kmajor ? (x.size(0) == N[p] && x.size(1) == R) : (x.size(0) == R && x.size(1) == N[p]),
                    "gemm_pp_dw_group: X shape mismatch");
        TORCH_CHECK(gemm_pp_shape_ok(M[p], N[p], R, (int)splits),
                    "gemm_pp_dw_group: M, N must be multiples of 256, R of 64 (>= splits)");
        TORCH_CHECK(dy.stride(0) % 8 == 0 && x.stride(0) % 8 == 0 && g.stride(0) % 8 == 0,
                    "gemm_pp_dw_group: 16-byte row alignment");
        TORCH_CHECK(dy.stride(0) * 256 < (1L << 31) && x.stride(0) * 256 < (1L << 31),
                    "gemm_pp_dw_group: leading dimension too large for 32-bit tile offsets");
        A[p] = dy.data_ptr();
        B[p] = x.data_ptr();
        C[p] = g.data_ptr();
        lda[p] = dy.stride(0);
        ldb[p] = x.stride(0);
        ldc[p] = g.stride(0);
        slab_elems += splits * (long)M[p] * N[p];
    }
    DevGuard dg(gs[0].device());
    auto slab = at::empty({slab_elems}, gs[0].options().dtype(at::kFloat));
    launch_gemm_pp_dw_group(np, A, lda, B, ldb, x_kmajor ? 1 : 0, C, ldc, M, N, R, (int)splits, (float)beta,
                            slab.data_ptr<float>(), c32 ? 1 : 0, cur_stream());
}

// y = (a8 @ b8^T) * sa * sb in bf16: a8 [M, K] e4m3 / e5m2, b8 [N, K] e4m3 (both K-major), sa / sb device fp32
// scalars (the per-tensor inverse scales); the hand-written fp8 MFMA ping-pong kernel (gemm_pp.hip)
at::Tensor gemm_fp8(const at::Tensor& a8, const at::Tensor& b8, const at::Tensor& sa, const at::Tensor& sb) {
    check_cuda(a8, "a8");
    check_cuda(b8, "b8");
    const bool a_e5 = a8.scalar_type() == at::kFloat8_e5m2;
    TORCH_CHECK((a8.scalar_type() == at::kFloat8_e4m3fn || a_e5) && b8.scalar_type() == at::kFloat8_e4m3fn,
                "gemm_fp8: a8 must be float8_e4m3fn or float8_e5m2, b8 float8_e4m3fn");
    TORCH_CHECK(a8.dim() == 2 && b8.dim() == 2 && a8.stride(1) == 1 && b8.stride(1) == 1 && a8.size(1) == b8.size(1),
                "gemm_fp8: a8 [M, K] and b8 [N, K] row-major with a common K");
    const int64_t M = a8.size(0), N = b8.size(0), K = a8.size(1);
    TORCH_CHECK(M % 256 == 0 && N % 256 == 0 && K % 128 == 0 && K > 0,
                "gemm_fp8: M, N must be multiples of 256 and K of 128");
    TORCH_CHECK(a8.stride(0) % 16 == 0 && b8.stride(0) % 16 == 0 && (a8.stride(0) * 256) < (1L << 32),
                "gemm_fp8: 16-byte aligned rows");
    TORCH_CHECK(sa.scalar_type() == at::kFloat && sb.scalar_type() == at::kFloat && sa.numel() >= 1 &&
                    sb.numel() >= 1 && sa.device() == a8.device() && sb.device() == a8.device(),
                "gemm_fp8: sa / sb must be fp32 device scalars");
    DevGuard g(a8.device());
    auto y = at::empty({M, N}, a8.options().dtype(at::kBFloat16));
    launch_gemm_fp8(a8.data_ptr(), a8.stride(0), b8.data_ptr(), b8.stride(0), y.data_ptr(), y.stride(0), (int)M,
                    (int)N, (int)K, a_e5 ? 1 : 0, sa.data_ptr<float>(), sb.data_ptr<float>(), cur_stream());
    return y;
}

// gu = (x8 @ w8^T) * sa * sb (e4m3 x e4m3; w8 = [W1; W3] e4m3 [2F, K]) with a = silu(g) * u cast to e4m3 with
// a_scale in both layouts (a8 [M, F], a8t [F, M]) and max |a| folded into a_amax: the fp8 W13 GEMM and the
// swiglu_cast_fp8_t pass in one kernel (gemm_pp.hip EPI_SWIGLU_FWD8)
at::Tensor gemm_fp8_swiglu(const at::Tensor& x8, const at::Tensor& w8, const at::Tensor& sa, const at::Tensor& sb,
                           const at::Tensor& a_scale, at::Tensor a8, at::Tensor a8t, at::Tensor a_amax) {
    check_cuda(x8, "x8");
    check_cuda(w8, "w8");
    TORCH_CHECK(x8.scalar_type() == at::kFloat8_e4m3fn && w8.scalar_type() == at::kFloat8_e4m3fn,
                "gemm_fp8_swiglu: e4m3 operands");
    TORCH_CHECK(x8.dim() == 2 && w8.dim() == 2 && x8.is_contiguous() && w8.is_contiguous() && x8.size(1) == w8.size(1),
                "gemm_fp8_swiglu: x8 [M, K] and w8 [2F, K] contiguous with a common K");
    const int64_t M = x8.size(0), F = w8.size(0) / 2, K = x8.size(1);
    TORCH_CHECK(w8.size(0) == 2 * F && M % 256 == 0 && F % 128 == 0 && K % 128 == 0 && K > 0,
                "gemm_fp8_swiglu: M a multiple of 256, F of 128, K of 128");
    TORCH_CHECK(K * 256 < (1L << 32) && 2 * F * K < (1L << 32), "gemm_fp8_swiglu: operand offsets exceed 32 bits");
    TORCH_CHECK(a8.is_contiguous() && a8t.is_contiguous() && a8.scalar_type() == at::kFloat8_e4m3fn &&
                    a8t.scalar_type() == at::kFloat8_e4m3fn && a8.dim() == 2 && a8.size(0) == M && a8.size(1) == F &&
                    a8t.dim() == 2 && a8t.size(0) == F && a8t.size(1) == M && a8.device() == x8.device() &&
                    a8t.device() == x8.device(),
                "gemm_fp8_swiglu: a8 [M, F] and a8t [F, M] e4m3 on the operands' device");
    TORCH_CHECK(sa.scalar_type() == at::kFloat && sb.scalar_type() == at::kFloat && a_scale.scalar_type() == at::kFloat &&
                    sa.numel() >= 1 && sb.numel() >= 1 && a_scale.numel() == 1 && a_amax.scalar_type() == at::kInt &&
                    a_amax.numel() == 1 && sa.device() == x8.device() && sb.device() == x8.device() &&
                    a_scale.device() == x8.device() && a_amax.device() == x8.device(),
                "gemm_fp8_swiglu: fp32 device scalars sa, sb, a_scale and one int32 amax slot");
    DevGuard g(x8.device());
    auto gu = at::empty({M, 2 * F}, x8.options().dtype(at::kBFloat16));
    launch_gemm_fp8_swiglu(x8.data_ptr(), x8.stride(0), w8.data_ptr(), w8.stride(0), gu.data_ptr(), gu.stride(0),
                           a8.data_ptr(), a8t.data_ptr(), (int)M, (int)F, (int)K, sa.data_ptr<float>(),
                           sb.data_ptr<float>(), a_scale.data_ptr<float>(),
                           reinterpret_cast<unsigned*>(a_amax.data_ptr<int>()), cur_stream());
    return gu;
}

// the fp8 W2 input gradient with the SwiGLU backward fused: da = (g8 @ w8t^T) * sa * sb (g8 e5m2 [M, K], w8t e4m3
// [F, K]) never leaves the kernel; [dg | du] from da and gu ([M, 2F] bf16) is written as e5m2 with d_scale in both
// layouts (dgu8 [M, 2F], dgu8t [2F, M]) and its max folded into d_amax (gemm_pp.hip EPI_SWIGLU_BWD8)
void gemm_fp8_swiglu_bwd(const at::Tensor& g8, const at::Tensor& w8t, const at::Tensor& sa, const at::Tensor& sb,
                         const at::Tensor& gu, const at::Tensor& d_scale, at::Tensor dgu8, at::Tensor dgu8t,
                         at::Tensor d_amax) {
    check_cuda(g8, "g8");
    check_cuda(w8t, "w8t");
    check_cuda(gu, "gu");
    TORCH_CHECK(g8.scalar_type() == at::kFloat8_e5m2 && w8t.scalar_type() == at::kFloat8_e4m3fn,
                "gemm_fp8_swiglu_bwd: g8 e5m2, w8t e4m3");
    TORCH_CHECK(g8.dim() == 2 && w8t.dim() == 2 && g8.is_contiguous() && w8t.is_contiguous() && g8.size(1) == w8t.size(1),
                "gemm_fp8_swiglu_bwd: g8 [M, K] and w8t [F, K] contiguous with a common K");
    const int64_t M = g8.size(0), F = w8t.size(0), K = g8.size(1);
    TORCH_CHECK(M % 256 == 0 && F % 256 == 0 && K % 128 == 0 && K > 0,
                "gemm_fp8_swiglu_bwd: M and F multiples of 256, K of 128");
    TORCH_CHECK(K * 256 < (1L << 32) && F * K < (1L << 32), "gemm_fp8_swiglu_bwd: operand offsets exceed 32 bits");
    TORCH_CHECK(gu.scalar_type() == at::kBFloat16 && gu.is_contiguous() && gu.dim() == 2 && gu.size(0) == M &&
                    gu.size(1) == 2 * F && gu.device() == g8.device(), "gemm_fp8_swiglu_bwd: gu bf16 [M, 2F]");
    TORCH_CHECK(dgu8.is_contiguous() && dgu8t.is_contiguous() && dgu8.scalar_type() == at::kFloat8_e5m2 &&
                    dgu8t.scalar_type() == at::kFloat8_e5m2 && dgu8.dim() == 2 && dgu8.size(0) == M &&
                    dgu8.size(1) == 2 * F && dgu8t.dim() == 2 && dgu8t.size(0) == 2 * F && dgu8t.size(1) == M &&
                    dgu8.device() == g8.device() && dgu8t.device() == g8.device(),
                "gemm_fp8_swiglu_bwd: dgu8 [M, 2F] and dgu8t [2F, M] e5m2 on the operands' device");
    TORCH_CHECK(sa.scalar_type() == at::kFloat && sb.scalar_type() == at::kFloat && d_scale.scalar_type() == at::kFloat &&
                    sa.numel() >= 1 && sb.numel() >= 1 && d_scale.numel() == 1 && d_amax.scalar_type() == at::kInt &&
                    d_amax.numel() == 1 && sa.device() == g8.device() && sb.device() == g8.device() &&
                    d_scale.device() == g8.device() && d_amax.device() == g8.device(),
                "gemm_fp8_swiglu_bwd: fp32 device scalars sa, sb, d_scale and one int32 amax slot");
    DevGuard g(g8.device());
    launch_gemm_fp8_swiglu_bwd(g8.data_ptr(), g8.stride(0), w8t.data_ptr(), w8t.stride(0), gu.data_ptr(),
                               dgu8.data_ptr(), dgu8t.data_ptr(), (int)M, (int)F, (int)K, sa.data_ptr<float>(),
                               sb.data_ptr<float>(), d_scale.data_ptr<float>(),
                               reinterpret_cast<unsigned*>(d_amax.data_ptr<int>()), cur_stream());
}

// qkv = (a8 @ b8^T) * sa * sb (e4m3 x e4m3) with RoPE on output columns [0, rot_cols) in the epilogue
at::Tensor gemm_fp8_rope(const at::Tensor& a8, const at::Tensor& b8, const at::Tensor& sa, const at::Tensor& sb,
                         const at::Tensor& cos, const at::Tensor& sin, int64_t S, int64_t D, int64_t rot_cols) {
    check_cuda(a8, "a8");
    check_cuda(b8, "b8");
    TORCH_CHECK(a8.scalar_type() == at::kFloat8_e4m3fn && b8.scalar_type() == at::kFloat8_e4m3fn,
                "gemm_fp8_rope: e4m3 operands");
    TORCH_CHECK(a8.dim() == 2 && b8.dim() == 2 && a8.stride(1) == 1 && b8.stride(1) == 1 && a8.size(1) == b8.size(1),
                "gemm_fp8_rope: a8 [M, K] and b8 [N, K] row-major with a common K");
    const int64_t M = a8.size(0), N = b8.size(0), K = a8.size(1);
    TORCH_CHECK(M % 256 == 0 && N % 256 == 0 && K % 128 == 0 && K > 0, "gemm_fp8_rope: M, N multiples of 256, K of 128");
    TORCH_CHECK(a8.stride(0) % 16 == 0 && b8.stride(0) % 16 == 0 && (a8.stride(0) * 256) < (1L << 32),
                "gemm_fp8_rope: 16-byte aligned rows");
    TORCH_CHECK(sa.scalar_type() == at::kFloat && sb.scalar_type() == at::kFloat && sa.numel() >= 1 &&
                    sb.numel() >= 1 && sa.device() == a8.device() && sb.device() == a8.device(),
                "gemm_fp8_rope: sa / sb must be fp32 device scalars");
    TORCH_CHECK(D % 8 == 0 && rot_cols % D == 0 && rot_cols <= N && S > 0 && M % S == 0,
                "gemm_fp8_rope: D multiple of 8, rot_cols of D, rows a multiple of S");
    TORCH_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat && cos.is_contiguous() &&
                    sin.is_contiguous() && cos.device() == a8.device() && sin.device() == a8.device() &&
                    cos.numel() >= S * (D / 2) && sin.numel() >= S * (D / 2),
                "gemm_fp8_rope: contiguous fp32 cos / sin tables of >= S rows on the GPU");
    DevGuard g(a8.device());
    auto y = at::empty({M, N}, a8.options().dtype(at::kBFloat16));
    launch_gemm_fp8_rope(a8.data_ptr(), a8.stride(0), b8.data_ptr(), b8.stride(0), y.data_ptr(), y.stride(0), (int)M,
                         (int)N, (int)K, sa.data_ptr<float>(), sb.data_ptr<float>(), cos.data_ptr<float>(),
                         sin.data_ptr<float>(), (int)S, (int)D, (int)rot_cols, cur_stream());
    return y;
}

// c = beta * c + (a8 @ b8^T) * sa * sb, split-K (`splits` fp32 partials, ordered reduce): the fp8 weight-gradient
// GEMM, accumulating straight into the (bf16 or fp32) gradient buffer view c
void gemm_fp8_acc(const at::Tensor& a8, const at::Tensor& b8, const at::Tensor& sa, const at::Tensor& sb, at::Tensor c,
                  double beta, int64_t splits) {
    check_cuda(a8, "a8");
    check_cuda(c, "c");
    const bool a_e5 = a8.scalar_type() == at::kFloat8_e5m2;
    TORCH_CHECK((a8.scalar_type() == at::kFloat8_e4m3fn || a_e5) && b8.scalar_type() == at::kFloat8_e4m3fn,
                "gemm_fp8_acc: a8 must be float8_e4m3fn or float8_e5m2, b8 float8_e4m3fn");
    TORCH_CHECK(a8.dim() == 2 && b8.dim() == 2 && a8.stride(1) == 1 && b8.stride(1) == 1 && a8.size(1) == b8.size(1),
                "gemm_fp8_acc: a8 [M, K] and b8 [N, K] row-major with a common K");
    const int64_t M = a8.size(0), N = b8.size(0), K = a8.size(1);
    TORCH_CHECK(c.dim() == 2 && c.size(0) == M && c.size(1) == N && c.stride(1) == 1 &&
                    (c.scalar_type() == at::kBFloat16 || c.scalar_type() == at::kFloat),
                "gemm_fp8_acc: c [M, N] bf16 / fp32 with unit column stride");
    TORCH_CHECK(M % 256 == 0 && N % 256 == 0 && K % 128 == 0 && splits >= 1 && K / 128 >= splits,
                "gemm_fp8_acc: M, N multiples of 256, K of 128 (>= 128 x splits)");
    TORCH_CHECK(a8.stride(0) % 16 == 0 && b8.stride(0) % 16 == 0 && (a8.stride(0) * 256) < (1L << 32) &&
                    (b8.stride(0) * 256) < (1L << 32), "gemm_fp8_acc: 16-byte aligned rows, 32-bit tile offsets");
    TORCH_CHECK(sa.scalar_type() == at::kFloat && sb.scalar_type() == at::kFloat && sa.numel() >= 1 &&
                    sb.numel() >= 1 && sa.is_cuda() && sb.is_cuda(), "gemm_fp8_acc: sa / sb must be fp32 device scalars");
    DevGuard g(a8.device());
    auto slab = at::empty({splits, M, N}, c.options().dtype(at::kFloat));
    launch_gemm_fp8_splitk(a8.data_ptr(), a8.stride(0), b8.data_ptr(), b8.stride(0), c.data_ptr(), c.stride(0),
                           (int)M, (int)N, (int)K, a_e5 ? 1 : 0, sa.data_ptr<float>(), sb.data_ptr<float>(),
                           (float)beta, (int)splits, slab.data_ptr<float>(), c.scalar_type() == at::kFloat ? 1 : 0,
                           cur_stream());
}

// dgu = swiglu_bwd(dy @ w2, gu) with the SwiGLU backward in the GEMM epilogue (da never reaches HBM)
at::Tensor gemm_swiglu_bwd(const at::Tensor& dy, const at::Tensor& w2, const at::Tensor& gu) {
    check_cuda(gu, "gu");
    TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && w2.scalar_type() == at::kBFloat16 &&
                    gu.scalar_type() == at::kBFloat16, "gemm_swiglu_bwd: bf16 tensors required");
    TORCH_CHECK(dy.dim() == 2 && w2.dim() == 2 && gu.dim() == 2 && dy.stride(1) == 1 && w2.stride(1) == 1 &&
                    gu.is_contiguous(), "gemm_swiglu_bwd: row-major 2-D tensors required");
    const int M = (int)dy.size(0), R = (int)dy.size(1), F = (int)w2.size(1);
    TORCH_CHECK(w2.size(0) == R && gu.size(0) == M && gu.size(1) == 2 * F, "gemm_swiglu_bwd: shape mismatch");
    TORCH_CHECK(M % 256 == 0 && F % 256 == 0 && R % 64 == 0, "gemm_swiglu_bwd: M, F multiples of 256, d of 64");
    TORCH_CHECK(dy.stride(0) % 8 == 0 && w2.stride(0) % 8 == 0, "gemm_swiglu_bwd: 16-byte row alignment");
    DevGuard g(gu.device());
    auto dgu = at::empty_like(gu);
    launch_gemm_pp_swiglu_bwd(dy.data_ptr(), dy.stride(0), w2.data_ptr(), w2.stride(0), gu.data_ptr(),
                              dgu.data_ptr(), 2 * (long)F, M, F, R, cur_stream());
    return dgu;
}

// (gu, a): gu = x @ w13^T with a = silu(g) * u in the GEMM epilogue (no separate pass over gu)
std::tuple<at::Tensor, at::Tensor> gemm_swiglu_fwd(const at::Tensor& x, const at::Tensor& w13) {
    check_cuda(x, "x");
    TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w13.scalar_type() == at::kBFloat16,
                "gemm_swiglu_fwd: bf16 tensors required");
    TORCH_CHECK(x.dim() == 2 && w13.dim() == 2 && x.stride(1) == 1 && w13.stride(1) == 1,
                "gemm_swiglu_fwd: row-major 2-D tensors required");
    const int M = (int)x.size(0), R = (int)x.size(1), F = (int)(w13.size(0) / 2);
    TORCH_CHECK(w13.size(1) == R && w13.size(0) == 2 * F, "gemm_swiglu_fwd: shape mismatch");
    TORCH_CHECK(M % 256 == 0 && F % 128 == 0 && R % 64 == 0, "gemm_swiglu_fwd: M multiple of 256, F of 128, d of 64");
    TORCH_CHECK(x.stride(0) % 8 == 0 && w13.stride(0) % 8 == 0, "gemm_swiglu_fwd: 16-byte row alignment");
    TORCH_CHECK(2L * F * w13.stride(0) < (1L << 31) && 256L * x.stride(0) < (1L << 31),
                "gemm_swiglu_fwd: operand offsets exceed 32 bits");
    DevGuard g(x.device());
    auto gu = at::empty({M, 2 * F}, x.options());
    auto a = at::empty({M, F}, x.options());
    launch_gemm_pp_swiglu_fwd(x.data_ptr(), x.stride(0), w13.data_ptr(), w13.stride(0), gu.data_ptr(), 2 * (long)F,
                              a.data_ptr(), F, M, F, R, cur_stream());
    return {gu, a};
}

// qkv = x @ w^T with RoPE on its first rot_cols columns (Q and K heads, interleaved pairs, position = row % S)
// applied in the GEMM epilogue: the fused form of matmul + rope_qk_ (no second pass over Q / K)
at::Tensor gemm_qkv_rope(const at::Tensor& x, const at::Tensor& w, const at::Tensor& cos, const at::Tensor& sin,
                         int64_t S, int64_t D, int64_t rot_cols) {
    check_cuda(x, "x");
    TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16,
                "gemm_qkv_rope: bf16 operands required");
    TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.stride(1) == 1 && w.stride(1) == 1,
                "gemm_qkv_rope: row-major 2-D operands required");
    const int M = (int)x.size(0), R = (int)x.size(1), N = (int)w.size(0);
    TORCH_CHECK(w.size(1) == R, "gemm_qkv_rope: shape mismatch");
    TORCH_CHECK(M % 256 == 0 && N % 256 == 0 && R % 64 == 0, "gemm_qkv_rope: M, N multiples of 256, K of 64");
    TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0, "gemm_qkv_rope: 16-byte row alignment");
    TORCH_CHECK((long)N * w.stride(0) < (1L << 31) && 256L * x.stride(0) < (1L << 31),
                "gemm_qkv_rope: operand offsets exceed 32 bits");
    TORCH_CHECK(D % 8 == 0 && rot_cols % D == 0 && rot_cols <= N && S > 0 && M % S == 0,
                "gemm_qkv_rope: D multiple of 8, rot_cols of D, rows a multiple of S");
    TORCH_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat && cos.is_contiguous() &&
                    sin.is_contiguous() && cos.is_cuda() && sin.is_cuda(),
                "gemm_qkv_rope: contiguous fp32 cos / sin tables on the GPU required");
    TORCH_CHECK(cos.numel() >= S * (D / 2) && sin.numel() >= S * (D / 2), "gemm_qkv_rope: cos / sin shorter than S");
    DevGuard g(x.device());
    auto out = at::empty({M, N}, x.options());
    launch_gemm_pp_rope(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), N, M, N, R,
                        cos.data_ptr<float>(), sin.data_ptr<float>(), (int)S, (int)D, (int)rot_cols, cur_stream());
    return out;
}

// ---------------------------------------------------------------- FP8 quantisation (delayed scaling)
void cast_fp8(const at::Tensor& x, const at::Tensor& scale, at::Tensor out, at::Tensor amax_bits) {
    check_cuda(x, "x");
    TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && out.numel() == x.numel() && out.element_size() == 1,
                "cast_fp8: contiguous x and a same-size 1-byte output required");
    TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.numel() == 1, "cast_fp8: scale must be one fp32");
    TORCH_CHECK(amax_bits.scalar_type() == at::kInt && amax_bits.numel() == 1, "cast_fp8: amax slot must be int32");
    check_aligned(x, "x");
    DevGuard g(x.device());
    const int fmt = out.scalar_type() == at::kFloat8_e5m2 ? 1 : 0;
    TORCH_CHECK(fmt == 1 || out.scalar_type() == at::kFloat8_e4m3fn || out.scalar_type() == at::kByte,
                "cast_fp8: out must be float8_e4m3fn or float8_e5m2");
    launch_cast_fp8(dt_code(x), fmt, x.data_ptr(), x.numel(), scale.data_ptr<float>(), out.data_ptr(),
                    reinterpret_cast<unsigned*>(amax_bits.data_ptr<int>()), cur_stream());
}

// W [R][C] bf16 (row stride a multiple of 8) -> W^T [C][R] contiguous; scale (optional 0-dim / one-element fp32 device
// tensor): bf16(scale * W)^T
at::Tensor transpose_bf16(const at::Tensor& w, const std::optional<at::Tensor>& scale) {
    check_cuda(w, "w");
    TORCH_CHECK(w.dim() == 2 && w.scalar_type() == at::kBFloat16 && w.stride(1) == 1 && w.stride(0) % 8 == 0,
                "transpose_bf16: bf16 [R, C] with unit column stride and 16-byte row alignment required");
    const int64_t R = w.size(0), C = w.size(1);
    TORCH_CHECK(R % 64 == 0 && C % 64 == 0, "transpose_bf16: R and C must be multiples of 64");
    DevGuard g(w.device());
    const float* sp = nullptr;
    if (scale.has_value() && scale->defined()) {
        TORCH_CHECK(scale->scalar_type() == at::kFloat && scale->numel() == 1 && scale->device() == w.device(),
                    "transpose_bf16: scale must be a one-element fp32 tensor on w's device");
        sp = scale->data_ptr<float>();
    }
    auto out = at::empty({C, R}, w.options());
    launch_transpose_bf16(w.data_ptr(), w.stride(0), out.data_ptr(), R, (int)R, (int)C, cur_stream(), sp);
    return out;
}

// W [N][K] bf16 -> fp8 copies w8 [N][K] and w8t [K][N] in one pass (e4m3 or e5m2, both outputs the same format;
// amax folded into amax_bits)
void cast_fp8_t(const at::Tensor& w, const at::Tensor& scale, at::Tensor w8, at::Tensor w8t, at::Tensor amax_bits) {
    check_cuda(w, "w");
    TORCH_CHECK(w.dim() == 2 && w.is_contiguous() && w.scalar_type() == at::kBFloat16, "cast_fp8_t: bf16 [N, K]");
    const int N = (int)w.size(0), K = (int)w.size(1);
    TORCH_CHECK(N % 64 == 0 && K % 64 == 0, "cast_fp8_t: N and K must be multiples of 64");
    const bool e4 = w8.scalar_type() == at::kFloat8_e4m3fn, e5 = w8.scalar_type() == at::kFloat8_e5m2;
    TORCH_CHECK(w8.is_contiguous() && w8t.is_contiguous() && w8.numel() == w.numel() && w8t.numel() == w.numel() &&
                    (e4 || e5) && w8t.scalar_type() == w8.scalar_type() && w8t.size(0) == K,
                "cast_fp8_t: e4m3 or e5m2 outputs [N, K] and [K, N] of one format required");
    TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.numel() == 1 && amax_bits.scalar_type() == at::kInt &&
                    amax_bits.numel() == 1, "cast_fp8_t: one fp32 scale and one int32 amax slot");
    DevGuard g(w.device());
    launch_cast_fp8_t(w.data_ptr(), N, K, scale.data_ptr<float>(), w8.data_ptr(), w8t.data_ptr(),
                      reinterpret_cast<unsigned*>(amax_bits.data_ptr<int>()), e5 ? 1 : 0, cur_stream());
}

// SwiGLU with the two-layout fp8 cast fused: without dout, a = silu(g) u of gu = [g | u] [M, 2F] -> e4m3 o8 [M, F]
// and o8t [F, M]; with dout = dA [M, F], the gate gradient [dg | du] -> e5m2 o8 [M, 2F] and o8t [2F, M]
void swiglu_cast_fp8_t(const at::Tensor& gu, const c10::optional<at::Tensor>& dout, const at::Tensor& scale,
                       at::Tensor o8, at::Tensor o8t, at::Tensor amax_bits) {
    check_cuda(gu, "gu");
    TORCH_CHECK(gu.dim() == 2 && gu.is_contiguous() && gu.scalar_type() == at::kBFloat16, "swiglu_cast_fp8_t: bf16 gu");
    const int M = (int)gu.size(0), F = (int)(gu.size(1) / 2);
    TORCH_CHECK(gu.size(1) == 2 * F && M % 64 == 0 && F % 64 == 0, "swiglu_cast_fp8_t: M and F multiples of 64");
    const bool bwd = dout.has_value() && dout->defined();
    const int W = bwd ? 2 * F : F;
    if (bwd)
        TORCH_CHECK(dout->is_contiguous() && dout->scalar_type() == at::kBFloat16 && dout->size(0) == M &&
                        dout->size(1) == F && dout->device() == gu.device(), "swiglu_cast_fp8_t: dout bf16 [M, F]");
    const auto fmt = bwd ? at::kFloat8_e5m2 : at::kFloat8_e4m3fn;
    TORCH_CHECK(o8.is_contiguous() && o8t.is_contiguous() && o8.scalar_type() == fmt && o8t.scalar_type() == fmt &&
                    o8.dim() == 2 && o8.size(0) == M && o8.size(1) == W && o8t.dim() == 2 && o8t.size(0) == W &&
                    o8t.size(1) == M, "swiglu_cast_fp8_t: outputs [M, W] and [W, M] (e4m3 forward, e5m2 backward)");
    TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.numel() == 1 && amax_bits.scalar_type() == at::kInt &&
                    amax_bits.numel() == 1, "swiglu_cast_fp8_t: one fp32 scale and one int32 amax slot");
    DevGuard g(gu.device());
    launch_swiglu_cast_fp8_t(bwd ? 1 : 0, gu.data_ptr(), bwd ? dout->data_ptr() : nullptr, M, F,
                             scale.data_ptr<float>(), o8.data_ptr(), o8t.data_ptr(),
                             reinterpret_cast<unsigned*>(amax_bits.data_ptr<int>()), cur_stream());
}

// residual add + RMSNorm with an e4m3 output in both layouts: returns (sum, rstd); sum is empty without d (the
// caller's x is the norm input)
std::tuple<at::Tensor, at::Tensor> add_rmsnorm_cast_fp8_t(const at::Tensor& x, const c10::optional<at::Tensor>& d,
                                                          const at::Tensor& w, double eps, const at::Tensor& scale,
                                                          at::Tensor y8, at::Tensor y8t, at::Tensor amax_bits) {
    check_cuda(x, "x");
    TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && x.scalar_type() == at::kBFloat16, "add_rmsnorm_cast_fp8_t: bf16 x");
    const int M = (int)x.size(0), N = (int)x.size(1);
    TORCH_CHECK(M % 128 == 0 && N % 128 == 0 && N <= 2048, "add_rmsnorm_cast_fp8_t: M, N multiples of 128, N <= 2048");
    const bool add = d.has_value() && d->defined();
    if (add)
        TORCH_CHECK(d->is_contiguous() && d->scalar_type() == at::kBFloat16 && d->sizes() == x.sizes() &&
                        d->device() == x.device(), "add_rmsnorm_cast_fp8_t: d like x");
    TORCH_CHECK(w.is_contiguous() && w.scalar_type() == at::kBFloat16 && w.numel() == N, "add_rmsnorm_cast_fp8_t: w [N]");
    TORCH_CHECK(y8.is_contiguous() && y8t.is_contiguous() && y8.scalar_type() == at::kFloat8_e4m3fn &&
                    y8t.scalar_type() == at::kFloat8_e4m3fn && y8.size(0) == M && y8.size(1) == N &&
                    y8t.size(0) == N && y8t.size(1) == M, "add_rmsnorm_cast_fp8_t: e4m3 y8 [M, N] and y8t [N, M]");
    TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.numel() == 1 && amax_bits.scalar_type() == at::kInt &&
                    amax_bits.numel() == 1, "add_rmsnorm_cast_fp8_t: one fp32 scale and one int32 amax slot");
    DevGuard g(x.device());
    auto sum = add ? at::empty_like(x) : at::empty({0}, x.options());
    auto rstd = at::empty({M}, x.options().dtype(at::kFloat));
    launch_add_rmsnorm_cast_fp8_t(x.data_ptr(), add ? d->data_ptr() : nullptr, w.data_ptr(),
                                  add ? sum.data_ptr() : nullptr, y8.data_ptr(), y8t.data_ptr(), rstd.data_ptr<float>(),
                                  M, N, (float)eps, scale.data_ptr<float>(),
                                  reinterpret_cast<unsigned*>(amax_bits.data_ptr<int>()), cur_stream());
    return {sum, rstd};
}

void update_scales(at::Tensor amax_bits, at::Tensor hist, at::Tensor scale, at::Tensor inv_scale, int64_t pos,
                   double margin, int64_t fmt) {
    check_cuda(hist, "hist");
    const int n = (int)hist.size(0), H = (int)hist.size(1);
    TORCH_CHECK(amax_bits.numel() == n && scale.numel() == n && inv_scale.numel() == n, "update_scales: sizes");
    DevGuard g(hist.device());
    launch_update_scales(reinterpret_cast<unsigned*>(amax_bits.data_ptr<int>()), hist.data_ptr<float>(),
                         scale.data_ptr<float>(), inv_scale.data_ptr<float>(), n, H, (int)(pos % H), (float)margin,
                         (int)fmt, cur_stream());
}

// ---------------------------------------------------------------- RoPE
at::Tensor rope(const at::Tensor& x, const at::Tensor& pos, const at::Tensor& cos, const at::Tensor& sin,
                bool inverse) {
    check_cuda(x, "x");
    TORCH_CHECK(x.is_contiguous() && x.dim() == 3, "rope: x must be contiguous [R, H, D]");
    TORCH_CHECK(pos.scalar_type() == at::kLong && pos.numel() == x.size(0), "rope: pos must be int64 [R]");
    const int D = (int)x.size(2);
    TORCH_CHECK(D % vec_elems(x) == 0, "rope: head dim must be a multiple of 8 (bf16) / 4 (fp32)");
    TORCH_CHECK(cos.size(1) == D / 2 && cos.scalar_type() == at::kFloat, "rope: cos table must be fp32 [S, D/2]");
    DevGuard g(x.device());
    auto y = at::empty_like(x);
    auto p = pos.contiguous();
    launch_rope(dt_code(x), x.data_ptr(), y.data_ptr(), p.data_ptr<int64_t>(), cos.data_ptr<float>(),
                sin.data_ptr<float>(), x.size(0), (int)x.size(1), D, inverse ? 1 : 0, cur_stream());
    return y;
}

// ---------------------------------------------------------------- flash attention
void check_qkv(const at::Tensor& t, int64_t rows, int64_t cols, const char* name) {
    check_cuda(t, name);
    TORCH_CHECK(t.scalar_type() == at::kBFloat16, "flash attention: ", name, " must be bf16");
    TORCH_CHECK(t.dim() == 2 && t.size(0) == rows && t.size(1) == cols && t.stride(1) == 1, "flash attention: ",
                name, " must be a [B*S, heads*D] view with unit column stride");
    TORCH_CHECK(t.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "flash attention: ",
                name, " rows must be 16-byte aligned");
}

// In-place RoPE of the Q and K heads of a fused QKV activation [B*S, (H + 2 Hkv) * D] (positions 0..S-1 per
// sequence); attention then runs in rope mode 2 (pre-rotated inputs).
void rope_qk_(at::Tensor qkv, const at::Tensor& cos, const at::Tensor& sin, int64_t B, int64_t S, int64_t H,
              int64_t Hkv, int64_t D) {
    check_cuda(qkv, "qkv");
    TORCH_CHECK(qkv.scalar_type() == at::kBFloat16, "rope_qk_: bf16 qkv required");
    TORCH_CHECK(qkv.dim() == 2 && qkv.size(0) == B * S && qkv.size(1) >= (H + Hkv) * D && qkv.stride(1) == 1,
                "rope_qk_: qkv must be [B*S, >= (H + Hkv) * D] with unit column stride");
    TORCH_CHECK(qkv.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(qkv.data_ptr()) % 16 == 0 && D % 8 == 0,
                "rope_qk_: rows must be 16-byte aligned");
    TORCH_CHECK(cos.scalar_type() == at::kFloat && cos.dim() == 2 && cos.size(0) >= S && cos.size(1) == D / 2 &&
                    cos.is_contiguous() && sin.is_contiguous() && sin.sizes() == cos.sizes(),
                "rope_qk_: rope tables must be fp32 [>=S, D/2]");
    DevGuard g(qkv.device());
    launch_rope_qk(qkv.data_ptr(), qkv.stride(0), cos.data_ptr<float>(), sin.data_ptr<float>(), B * S, (int)S,
                   (int)H, (int)Hkv, (int)D, cur_stream());
}

// the fp32 dQ accumulator shared by fa_fwd (zeroes it) and fa_bwd: [B * Spad, H * D], Spad = S rounded up to 64
void check_dq_acc(const at::Tensor& t, const at::Tensor& q, int64_t B, int64_t S, int64_t H, int64_t D) {
    check_cuda(t, "dq_acc");
    TORCH_CHECK(t.scalar_type() == at::kFloat && t.is_contiguous() && t.dim() == 2 &&
                    t.size(0) == B * ((S + 63) / 64 * 64) && t.size(1) == H * D && t.device() == q.device(),
                "flash attention: dq_acc must be a contiguous fp32 [B * round_up(S, 64), H * D] tensor on q's device");
}

std::tuple<at::Tensor, at::Tensor> fa_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                          const at::Tensor& cos, const at::Tensor& sin, int64_t B, int64_t S, int64_t H,
                                          int64_t Hkv, int64_t D, bool causal, bool use_rope, double scale,
                                          bool prerotated, const c10::optional<at::Tensor>& dq_acc) {
    TORCH_CHECK(D == 64 || D == 128, "flash attention: head dim must be 64 or 128");
    TORCH_CHECK(H % Hkv == 0, "flash attention: H must be a multiple of Hkv");
    check_qkv(q, B * S, H * D, "q");
    check_qkv(k, B * S, Hkv * D, "k");
    check_qkv(v, B * S, Hkv * D, "v");
    TORCH_CHECK(k.stride(0) == v.stride(0), "flash attention: k and v must share a row stride");
    if (use_rope && !prerotated)
        TORCH_CHECK(cos.scalar_type() == at::kFloat && cos.size(0) >= S && cos.size(1) == D / 2 && cos.is_contiguous()
                        && sin.is_contiguous(), "flash attention: rope tables must be fp32 [>=S, D/2]");
    DevGuard g(q.device());
    auto o = at::empty({B * S, H * D}, q.options());
    auto lse = at::empty({B, H, S}, q.options().dtype(at::kFloat));
    FaArgs a{};
    a.q = (const __bf16*)q.data_ptr(); a.k = (const __bf16*)k.data_ptr(); a.v = (const __bf16*)v.data_ptr();
    a.ld_q = q.stride(0); a.ld_kv = k.stride(0);
    a.o = (__bf16*)o.data_ptr(); a.ld_o = H * D; a.lse = lse.data_ptr<float>();
    const bool fused_rope = use_rope && !prerotated;
    a.cos = fused_rope ? cos.data_ptr<float>() : nullptr; a.sin = fused_rope ? sin.data_ptr<float>() : nullptr;
    a.B = (int)B; a.H = (int)H; a.Hkv = (int)Hkv; a.S = (int)S; a.D = (int)D;
    a.causal = causal; a.rope = use_rope ? (prerotated ? 2 : 1) : 0; a.scale = (float)scale;
    if (dq_acc.has_value() && dq_acc->defined()) {  // training: the forward zeroes the backward's dQ accumulator
        check_dq_acc(*dq_acc, q, B, S, H, D);
        a.dq_acc = dq_acc->data_ptr<float>();
    }
    launch_fa_fwd(a, cur_stream());
    return {o, lse};
}

// whether fa_bwd uses (and fa_fwd should zero) the fp32 dQ accumulator for head dim D
bool fa_bwd_needs_dq_acc(int64_t D) { return !fa_bwd_split_active((int)D, 2); }
int64_t fa_fwd_config_op(int64_t ver) { return fa_fwd_config((int)ver); }
int64_t fa_bwd_config_op(int64_t mode) { return fa_bwd_config((int)mode); }
int64_t fa_dq_config_op(int64_t form) { return fa_dq_config((int)form); }
int64_t gpp_persist_config_op(int64_t mode) { return gpp_persist_config((int)mode); }
int64_t gpp_order_config_op(int64_t gm) { return gpp_order_config((int)gm); }
// [n, 8] int64 stamps of the last split-backward kernel (a BPE_FA_STAMPS variant build), or an empty tensor
at::Tensor fa_stamps_op(int64_t n) {
    auto t = at::empty({n, 8}, at::TensorOptions().dtype(at::kLong));
    if (!fa_read_stamps(reinterpret_cast<long long*>(t.data_ptr<int64_t>()), (int)n)) return at::empty({0, 8}, t.options());
    return t;
}
// the same for the last gemm_pp kernel (a BPE_GPP_STAMPS variant build)
// phase stamps (BPE_GPP_PHASE_STAMPS builds): [n workgroups][8 waves][4 K-tiles][4 phases][4 events]
at::Tensor gpp_phase_stamps_op(int64_t n) {
    auto t = at::empty({n, 8, 4, 4, 4}, at::TensorOptions().dtype(at::kLong));
    if (!gpp_read_phase_stamps(reinterpret_cast<long long*>(t.data_ptr<int64_t>()), (int)n))
        return at::empty({0, 8, 4, 4, 4}, t.options());
    return t;
}

at::Tensor gpp_stamps_op(int64_t n) {
    auto t = at::empty({n, 8}, at::TensorOptions().dtype(at::kLong));
    if (!gpp_read_stamps(reinterpret_cast<long long*>(t.data_ptr<int64_t>()), (int)n)) return at::empty({0, 8}, t.options());
    return t;
}


// Returns dqkv = [B*S, (H + 2*Hkv) * D]: dq | dk | dv in the fused QKV-projection layout.
at::Tensor fa_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                  const at::Tensor& o, const at::Tensor& lse, const at::Tensor& cos, const at::Tensor& sin, int64_t B,
                  int64_t S, int64_t H, int64_t Hkv, int64_t D, bool causal, bool use_rope, double scale,
                  bool prerotated, const c10::optional<at::Tensor>& dq_acc_in) {
    TORCH_CHECK(D == 64 || D == 128, "flash attention: head dim must be 64 or 128");
    TORCH_CHECK(Hkv > 0 && H % Hkv == 0, "flash attention: H must be a multiple of Hkv");
    if (use_rope)
        TORCH_CHECK(cos.scalar_type() == at::kFloat && cos.size(0) >= S && cos.size(1) == D / 2 && cos.is_contiguous()
                        && sin.is_contiguous(), "flash attention: rope tables must be fp32 [>=S, D/2]");
    check_qkv(q, B * S, H * D, "q");
    check_qkv(k, B * S, Hkv * D, "k");
    check_qkv(v, B * S, Hkv * D, "v");
    auto d = dout.contiguous();
    check_qkv(d, B * S, H * D, "dout");
    check_qkv(o, B * S, H * D, "o");
    DevGuard g(q.device());
    const int64_t W = (H + 2 * Hkv) * D;
    auto dqkv = at::empty({B * S, W}, q.options());
    auto delta = at::empty({B, H, S}, q.options().dtype(at::kFloat));
    int rope = use_rope ? (prerotated ? 2 : 1) : 0;
    // D = 128 with the forward's in-kernel rotation: the split kernels take pre-rotated Q / K, so rotate a copy of
    // [Q | K | V] (the kernels then un-rotate dQ / dK on output, as for the pre-rotated forward)
    at::Tensor qkv_rot;
    const __bf16 *qp = (const __bf16*)q.data_ptr(), *kp = (const __bf16*)k.data_ptr(), *vp = (const __bf16*)v.data_ptr();
    int64_t ld_q = q.stride(0), ld_kv = k.stride(0);
    if (D == 128 && rope == 1 && fa_bwd_split_active((int)D, 2)) {
        TORCH_CHECK(k.stride(0) == v.stride(0), "flash attention: k and v must share a row stride");
        qkv_rot = at::cat({q, k, v}, 1);
        launch_rope_qk(qkv_rot.data_ptr(), W, cos.data_ptr<float>(), sin.data_ptr<float>(), B * S, (int)S, (int)H,
                       (int)Hkv, (int)D, cur_stream());
        qp = (const __bf16*)qkv_rot.data_ptr();
        kp = qp + H * D;
        vp = qp + (H + Hkv) * D;
        ld_q = ld_kv = W;
        rope = 2;
    }
    // rows padded to 64 per batch; zeroed by the forward when it was handed this buffer (fa_fwd dq_acc)
    const bool split = fa_bwd_split_active((int)D, rope);  // the split form needs no fp32 dQ accumulator
    const bool pre_zeroed = !split && dq_acc_in.has_value() && dq_acc_in->defined();
    if (pre_zeroed) check_dq_acc(*dq_acc_in, q, B, S, H, D);
    at::Tensor dq_acc;
    if (!split)
        dq_acc = pre_zeroed ? *dq_acc_in : at::empty({B * ((S + 63) / 64 * 64), H * D}, q.options().dtype(at::kFloat));
    at::Tensor dkv_part;
    const bool need_part = Hkv < H && fa_dkv_partials_needed((int)D, rope);  // GQA per-query-head partials (+ reduce)
    if (need_part) dkv_part = at::empty({B * S, H * 2 * D}, q.options().dtype(at::kFloat));
    FaArgs a{};
    a.q = qp; a.k = kp; a.v = vp;
    a.ld_q = ld_q; a.ld_kv = ld_kv;
    a.o = (__bf16*)o.data_ptr(); a.ld_o = o.stride(0); a.lse = lse.data_ptr<float>();
    a.cos = use_rope ? cos.data_ptr<float>() : nullptr; a.sin = use_rope ? sin.data_ptr<float>() : nullptr;
    a.B = (int)B; a.H = (int)H; a.Hkv = (int)Hkv; a.S = (int)S; a.D = (int)D;
    a.causal = causal; a.rope = rope; a.scale = (float)scale;
    a.dout = (const __bf16*)d.data_ptr(); a.ld_do = d.stride(0);
    a.delta = delta.data_ptr<float>(); a.dq_acc = split ? nullptr : dq_acc.data_ptr<float>();
    a.dq_zeroed = pre_zeroed ? 1 : 0;
    __bf16* base = (__bf16*)dqkv.data_ptr();
    a.dq = base; a.ld_dq = W;
    a.dk = base + H * D; a.dv = base + (H + Hkv) * D; a.ld_dkv = W;
    a.dkv_part = need_part ? dkv_part.data_ptr<float>() : nullptr;
    launch_fa_bwd(a, cur_stream());
    return dqkv;
}

// ---------------------------------------------------------------- KV-cache decode (serving)
void check_cache(const at::Tensor& c, int64_t B, int64_t Hkv, const char* name) {
    check_cuda(c, name);
    TORCH_CHECK(c.scalar_type() == at::kBFloat16 && c.dim() == 4 && c.is_contiguous(), "kv cache: ", name,
                " must be a contiguous bf16 [B, Hkv, Lmax, D] tensor");
    TORCH_CHECK(c.size(0) == B && c.size(1) == Hkv, "kv cache: ", name, " batch / kv-head mismatch");
    check_aligned(c, name);
}

void check_pos(const at::Tensor& pos) {
    check_cuda(pos, "pos");
    TORCH_CHECK(pos.scalar_type() == at::kInt && pos.numel() == 1, "kv cache: pos must be one device int32");
}

// qkv [B*T, (H + 2*Hkv)*D] rows of T new tokens at positions *pos.. -> roped q [B*T, H*D]; K (roped) and V are
// written into the caches at those positions.
at::Tensor kv_append(const at::Tensor& qkv, at::Tensor kc, at::Tensor vc, const at::Tensor& cos, const at::Tensor& sin,
                     const at::Tensor& pos, int64_t B, int64_t T, int64_t H, bool use_rope) {
    const int64_t Hkv = kc.size(1), Lmax = kc.size(2), D = kc.size(3);
    TORCH_CHECK(D % 8 == 0 && H % Hkv == 0, "kv_append: head dim multiple of 8, H multiple of Hkv");
    check_qkv(qkv, B * T, (H + 2 * Hkv) * D, "qkv");
    check_cache(kc, B, Hkv, "k_cache");
    check_cache(vc, B, Hkv, "v_cache");
    TORCH_CHECK(vc.sizes() == kc.sizes(), "kv_append: k / v cache shapes differ");
    check_pos(pos);
    if (use_rope)
        TORCH_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat && cos.is_contiguous() &&
                        sin.is_contiguous() && cos.size(0) >= Lmax && cos.size(1) == D / 2 && sin.sizes() == cos.sizes(),
                    "kv_append: rope tables must be fp32 [>=Lmax, D/2]");
    DevGuard g(qkv.device());
    auto q = at::empty({B * T, H * D}, qkv.options());
    launch_kv_append(qkv.data_ptr(), qkv.stride(0), q.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                     use_rope ? cos.data_ptr<float>() : nullptr, use_rope ? sin.data_ptr<float>() : nullptr,
                     pos.data_ptr<int>(), (int)B, (int)T, (int)H, (int)Hkv, (int)D, (int)Lmax, cur_stream());
    return q;
}

// q [B, H*D] (roped) attends to the first *pos + 1 cache rows -> [B, H*D]
// combine = false: return the split partials [B*T, H, nsplit, D + 2] (o, m, l) for decode_attn_proj instead.
// T new tokens per sequence (q rows b * T + t, already appended at positions *pos .. *pos + T - 1).
at::Tensor decode_attn(const at::Tensor& q, const at::Tensor& kc, const at::Tensor& vc, const at::Tensor& pos,
                       int64_t H, double scale, bool combine, int64_t T) {
    const int64_t B = kc.size(0), Hkv = kc.size(1), Lmax = kc.size(2), D = kc.size(3);
    TORCH_CHECK(decode_attn_ok((int)H, (int)Hkv, (int)D, (int)T),
                "decode_attn: head dim 64/128, H a multiple of Hkv and (H / Hkv) * T <= 8 required");
    check_cuda(q, "q");
    TORCH_CHECK(q.scalar_type() == at::kBFloat16 && q.is_contiguous() && q.numel() == B * T * H * D,
                "decode_attn: q must be contiguous bf16 [B*T, H*D]");
    check_cache(kc, B, Hkv, "k_cache");
    check_cache(vc, B, Hkv, "v_cache");
    TORCH_CHECK(vc.sizes() == kc.sizes(), "decode_attn: k / v cache shapes differ");
    check_pos(pos);
    DevGuard g(q.device());
    const int ns = decode_attn_splits((int)Lmax);
    auto part = at::empty({B * T, H, ns, D + 2}, q.options().dtype(at::kFloat));
    auto out = combine ? at::empty({B * T, H * D}, q.options()) : at::Tensor();
    launch_decode_attn(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), part.data_ptr<float>(),
                       combine ? out.data_ptr() : nullptr, pos.data_ptr<int>(), (int)B, (int)T, (int)H, (int)Hkv,
                       (int)D, (int)Lmax, (float)scale, cur_stream());
    return combine ? out : part;
}

// Skinny-GEMM prologue / shape checks shared by decode_gemv and decode_qkv; returns the residual-sum output
at::Tensor gemv_setup(GemvArgs& a, const at::Tensor& x, const c10::optional<at::Tensor>& xd,
                      const c10::optional<at::Tensor>& ln, double eps, const at::Tensor& w) {
    check_cuda(x, "x");
    TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "decode gemv: bf16 required");
    TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "decode gemv: x must be [M, K] row-major");
    TORCH_CHECK(w.dim() == 2 && w.stride(1) == 1 && w.stride(0) % 8 == 0 && w.size(1) == x.size(1),
                "decode gemv: weight must be row-major [N, K]");
    const int M = (int)x.size(0), K = (int)x.size(1);
    TORCH_CHECK(gemv_ok(M, K), "decode gemv: 1 <= M <= 8 rows (<= 16 with K % 32 == 0) and K % 8 == 0 required");
    check_aligned(x, "x");
    check_aligned(w, "w");
    a = GemvArgs{};
    a.x = (const __bf16*)x.data_ptr();
    a.ldx = x.stride(0);
    a.W = (const __bf16*)w.data_ptr();
    a.ldw = w.stride(0);
    a.N = (int)w.size(0);
    a.K = K;
    a.M = M;
    a.eps = (float)eps;
    at::Tensor xsum = at::empty({0}, x.options());  // empty unless a residual sum is produced
    if (xd.has_value() && xd->defined()) {
        TORCH_CHECK(xd->sizes() == x.sizes() && xd->strides() == x.strides() && xd->scalar_type() == x.scalar_type(),
                    "decode gemv: xd must match x");
        check_aligned(*xd, "xd");
        a.xd = (const __bf16*)xd->data_ptr();
        xsum = at::empty({M, K}, x.options());
        a.xsum = (__bf16*)xsum.data_ptr();
    }
    if (ln.has_value() && ln->defined()) {
        TORCH_CHECK(ln->numel() == K && ln->is_contiguous() && ln->scalar_type() == at::kBFloat16,
                    "decode gemv: norm weight must be bf16 [K]");
        a.ln = (const __bf16*)ln->data_ptr();
    }
    return xsum;
}

// y = RMSNorm(x (+ xd)) W^T (epi 0) or SwiGLU over [W1; W3] (epi 1); returns (y, x + xd or an empty tensor)
std::tuple<at::Tensor, at::Tensor> decode_gemv(const at::Tensor& x, const c10::optional<at::Tensor>& xd,
                                               const c10::optional<at::Tensor>& ln, double eps, const at::Tensor& w,
                                               int64_t epi) {
    TORCH_CHECK(epi == 0 || epi == 1, "decode_gemv: epi must be 0 (plain) or 1 (SwiGLU)");
    GemvArgs a;
    auto xsum = gemv_setup(a, x, xd, ln, eps, w);
    TORCH_CHECK(epi == 0 || a.N % 2 == 0, "decode_gemv: SwiGLU needs an even number of rows");
    DevGuard g(x.device());
    auto y = at::empty({(int64_t)a.M, epi == 1 ? a.N / 2 : a.N}, x.options());
    a.y = (__bf16*)y.data_ptr();
    a.ldy = y.stride(0);
    launch_gemv(a, (int)epi, cur_stream());
    return {y, xsum};
}

// output projection of the decode attention straight from its split partials: y = combine(part) W^T
at::Tensor decode_attn_proj(const at::Tensor& part, const at::Tensor& w) {
    check_cuda(part, "part");
    TORCH_CHECK(part.scalar_type() == at::kFloat && part.dim() == 4 && part.is_contiguous(),
                "decode_attn_proj: part must be the fp32 [B, H, nsplit, D + 2] partials of decode_attn");
    const int64_t B = part.size(0), H = part.size(1), ns = part.size(2), D = part.size(3) - 2;
    TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.dim() == 2 && w.stride(1) == 1 && w.stride(0) % 8 == 0 &&
                    w.size(1) == H * D, "decode_attn_proj: weight must be row-major bf16 [N, H*D]");
    TORCH_CHECK(D % 8 == 0 && gemv_ok((int)B, (int)(H * D)), "decode_attn_proj: 1 <= B <= 16 and D % 8 == 0");
    check_aligned(w, "w");
    DevGuard g(part.device());
    GemvArgs a{};
    a.part = part.data_ptr<float>();
    a.nsplit = (int)ns;
    a.H = (int)H;
    a.D = (int)D;
    a.W = (const __bf16*)w.data_ptr();
    a.ldw = w.stride(0);
    a.N = (int)w.size(0);
    a.K = (int)(H * D);
    a.M = (int)B;
    auto y = at::empty({B, a.N}, w.options());
    a.y = (__bf16*)y.data_ptr();
    a.ldy = y.stride(0);
    launch_gemv(a, 0, cur_stream());
    return y;
}

// fused QKV projection for one new token per sequence: q (roped) out, K (roped) / V written into the caches
std::tuple<at::Tensor, at::Tensor> decode_qkv(const at::Tensor& x, const c10::optional<at::Tensor>& xd,
                                              const c10::optional<at::Tensor>& ln, double eps, const at::Tensor& w,
                                              at::Tensor kc, at::Tensor vc, const at::Tensor& cos,
                                              const at::Tensor& sin, const at::Tensor& pos, int64_t H, bool use_rope) {
    GemvArgs a;
    auto xsum = gemv_setup(a, x, xd, ln, eps, w);
    const int64_t B = a.M, Hkv = kc.size(1), Lmax = kc.size(2), D = kc.size(3);
    check_cache(kc, B, Hkv, "k_cache");
    check_cache(vc, B, Hkv, "v_cache");
    TORCH_CHECK(vc.sizes() == kc.sizes(), "decode_qkv: k / v cache shapes differ");
    TORCH_CHECK(a.N == (H + 2 * Hkv) * D && D % 2 == 0, "decode_qkv: weight rows must be (H + 2*Hkv) * D");
    check_pos(pos);
    if (use_rope)
        TORCH_CHECK(cos.scalar_type() == at::kFloat && cos.is_contiguous() && sin.is_contiguous() &&
                        cos.size(0) >= Lmax && cos.size(1) == D / 2 && sin.sizes() == cos.sizes(),
                    "decode_qkv: rope tables must be fp32 [>=Lmax, D/2]");
    DevGuard g(x.device());
    auto q = at::empty({B, H * D}, x.options());
    a.y = (__bf16*)q.data_ptr();
    a.ldy = q.stride(0);
    a.H = (int)H;
    a.Hkv = (int)Hkv;
    a.D = (int)D;
    a.Lmax = (int)Lmax;
    a.cosT = use_rope ? cos.data_ptr<float>() : nullptr;
    a.sinT = use_rope ? sin.data_ptr<float>() : nullptr;
    a.pos = pos.data_ptr<int>();
    a.kc = (__bf16*)kc.data_ptr();
    a.vc = (__bf16*)vc.data_ptr();
    launch_gemv(a, 2, cur_stream());
    return {q, xsum};
}

}  // namespace

TORCH_LIBRARY(bpe_hip, m) {
    m.def("decode_gemv(Tensor x, Tensor? xd, Tensor? ln, float eps, Tensor w, int epi) -> (Tensor, Tensor)");
    m.def("decode_qkv(Tensor x, Tensor? xd, Tensor? ln, float eps, Tensor w, Tensor(a!) k_cache, "
          "Tensor(b!) v_cache, Tensor cos, Tensor sin, Tensor pos, int H, bool rope) -> (Tensor, Tensor)");
    m.def("kv_append(Tensor qkv, Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor cos, Tensor sin, Tensor pos, int B, "
          "int T, int H, bool rope) -> Tensor");
    m.def("decode_attn(Tensor q, Tensor k_cache, Tensor v_cache, Tensor pos, int H, float scale, "
          "bool combine=True, int T=1) -> Tensor");
    m.def("decode_attn_proj(Tensor part, Tensor w) -> Tensor");
    m.def("rmsnorm_fwd(Tensor x, Tensor w, float eps) -> (Tensor, Tensor)");
    m.def("add_rmsnorm_fwd(Tensor x, Tensor d, Tensor w, float eps) -> (Tensor, Tensor, Tensor)");
    m.def("rmsnorm_bwd(Tensor dy, Tensor x, Tensor w, Tensor rstd, Tensor? dres=None, Tensor(a!)? dw_acc=None) -> "
          "(Tensor, Tensor)");
    m.def("swiglu_fwd(Tensor gu) -> Tensor");
    m.def("swiglu_bwd(Tensor dout, Tensor gu) -> Tensor");
    m.def("act_fwd(Tensor x, int kind) -> Tensor");
    m.def("act_bwd(Tensor dy, Tensor x, int kind) -> Tensor");
    m.def("ce_fwd_bwd(Tensor(a!) logits, Tensor targets, int ignore_index, bool write_grad, Tensor? nvalid=None) "
          "-> (Tensor, Tensor)");
    m.def("embed_fwd(Tensor weight, Tensor ids) -> Tensor");
    m.def("embed_bwd(Tensor dout, Tensor ids, int vocab) -> Tensor");
    m.def("adamw_step(Tensor(a!) p, Tensor(b!) m, Tensor(c!) v, Tensor grad, Tensor(d!)? pout, float lr, float b1, "
          "float b2, float eps, float wd, float bc1, float bc2_sqrt, Tensor? gscale, Tensor? nstep=None, "
          "Tensor? wd_mask=None) -> ()");
    m.def("adam_count_step(Tensor(a!) nstep, Tensor? gscale) -> ()");
    m.def("grad_norm(Tensor[] tensors, float max_norm) -> (Tensor, Tensor)");
    m.def("scale_(Tensor(a!) x, Tensor coef) -> ()");
    m.def("gemm_swiglu_bwd(Tensor dy, Tensor w2, Tensor gu) -> Tensor");
    m.def("gemm_swiglu_fwd(Tensor x, Tensor w13) -> (Tensor, Tensor)");
    m.def("gemm_qkv_rope(Tensor x, Tensor w, Tensor cos, Tensor sin, int S, int D, int rot_cols) -> Tensor");
    m.def("gemm_fp8_acc(Tensor a8, Tensor b8, Tensor sa, Tensor sb, Tensor(a!) c, float beta, int splits) -> ()");
    m.def("gemm_fp8(Tensor a8, Tensor b8, Tensor sa, Tensor sb) -> Tensor");
    m.def("gemm_fp8_swiglu(Tensor x8, Tensor w8, Tensor sa, Tensor sb, Tensor a_scale, Tensor(a!) a8, Tensor(b!) a8t, "
          "Tensor(c!) a_amax) -> Tensor");
    m.def("gemm_fp8_swiglu_bwd(Tensor g8, Tensor w8t, Tensor sa, Tensor sb, Tensor gu, Tensor d_scale, "
          "Tensor(a!) dgu8, Tensor(b!) dgu8t, Tensor(c!) d_amax) -> ()");
    m.def("gemm_fp8_rope(Tensor a8, Tensor b8, Tensor sa, Tensor sb, Tensor cos, Tensor sin, int S, int D, "
          "int rot_cols) -> Tensor");
    m.def("gemm_pp(Tensor A, bool a_kmajor, Tensor B, bool b_kmajor, Tensor(a!) C, float beta, int splits=1) -> ()");
    m.def("gemm_pp_dw_group(Tensor(a!)[] gs, Tensor[] dys, Tensor[] xs, bool x_kmajor, int splits, float beta=1.0) -> ()");
    m.def("gemm(Tensor A, bool a_kmajor, Tensor B, bool b_kmajor, Tensor(a!) C, float beta, int splits, int tile=128) -> ()");
    m.def("cast_fp8(Tensor x, Tensor scale, Tensor(a!) out, Tensor(b!) amax_bits) -> ()");
    m.def("transpose_bf16(Tensor w, Tensor? scale=None) -> Tensor");
    m.def("cast_fp8_t(Tensor w, Tensor scale, Tensor(a!) w8, Tensor(b!) w8t, Tensor(c!) amax_bits) -> ()");
    m.def("swiglu_cast_fp8_t(Tensor gu, Tensor? dout, Tensor scale, Tensor(a!) o8, Tensor(b!) o8t, "
          "Tensor(c!) amax_bits) -> ()");
    m.def("add_rmsnorm_cast_fp8_t(Tensor x, Tensor? d, Tensor w, float eps, Tensor scale, Tensor(a!) y8, "
          "Tensor(b!) y8t, Tensor(c!) amax_bits) -> (Tensor, Tensor)");
    m.def("update_scales(Tensor(a!) amax_bits, Tensor(b!) hist, Tensor(c!) scale, Tensor(d!) inv_scale, int pos, "
          "float margin, int fmt=0) -> ()");
    m.def("masked_sdpa(Tensor q, Tensor k, Tensor v, Tensor? mask, float scale) -> Tensor");
    m.def("softmax_fwd(Tensor x) -> Tensor");
    m.def("softmax_bwd(Tensor dy, Tensor y) -> Tensor");
    m.def("rope(Tensor x, Tensor pos, Tensor cos, Tensor sin, bool inverse) -> Tensor");
    m.def("fa_fwd(Tensor q, Tensor k, Tensor v, Tensor cos, Tensor sin, int B, int S, int H, int Hkv, int D, "
          "bool causal, bool rope, float scale, bool prerotated=False, Tensor? dq_acc=None) -> (Tensor, Tensor)");
    m.def("fa_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor cos, Tensor sin, int B, "
          "int S, int H, int Hkv, int D, bool causal, bool rope, float scale, bool prerotated=False, "
          "Tensor? dq_acc=None) -> Tensor");
    m.def("rope_qk_(Tensor(a!) qkv, Tensor cos, Tensor sin, int B, int S, int H, int Hkv, int D) -> ()");
    m.def("fa_bwd_needs_dq_acc(int D) -> bool", &fa_bwd_needs_dq_acc);  // no tensors: a catch-all kernel
    m.def("fa_bwd_config(int mode=-1) -> int", &fa_bwd_config_op);
    m.def("fa_dq_config(int form=-1) -> int", &fa_dq_config_op);
    m.def("fa_stamps(int n) -> Tensor", &fa_stamps_op);
    m.def("gpp_stamps(int n) -> Tensor", &gpp_stamps_op);
    m.def("gpp_phase_stamps(int n) -> Tensor", &gpp_phase_stamps_op);
    m.def("gpp_persist_config(int mode=-1) -> int", &gpp_persist_config_op);
    m.def("gpp_order_config(int gm=-1) -> int", &gpp_order_config_op);
    m.def("fa_fwd_config(int ver=0) -> int", &fa_fwd_config_op);
}

TORCH_LIBRARY_IMPL(bpe_hip, CUDA, m) {
    m.impl("rmsnorm_fwd", &rmsnorm_fwd);
    m.impl("add_rmsnorm_fwd", &add_rmsnorm_fwd);
    m.impl("rmsnorm_bwd", &rmsnorm_bwd);
    m.impl("swiglu_fwd", &swiglu_fwd);
    m.impl("swiglu_bwd", &swiglu_bwd);
    m.impl("act_fwd", &act_fwd);
    m.impl("act_bwd", &act_bwd);
    m.impl("ce_fwd_bwd", &ce_fwd_bwd);
    m.impl("embed_fwd", &embed_fwd);
    m.impl("embed_bwd", &embed_bwd);
    m.impl("adamw_step", &adamw_step);
    m.impl("adam_count_step", &adam_count_step);
    m.impl("grad_norm", &grad_norm);
    m.impl("scale_", &scale_);
    m.impl("gemm", &gemm);
    m.impl("gemm_pp", &gemm_pp);
    m.impl("gemm_pp_dw_group", &gemm_pp_dw_group);
    m.impl("gemm_swiglu_bwd", &gemm_swiglu_bwd);
    m.impl("gemm_swiglu_fwd", &gemm_swiglu_fwd);
    m.impl("gemm_qkv_rope", &gemm_qkv_rope);
    m.impl("gemm_fp8_acc", &gemm_fp8_acc);
    m.impl("gemm_fp8", &gemm_fp8);
    m.impl("gemm_fp8_swiglu", &gemm_fp8_swiglu);
    m.impl("gemm_fp8_swiglu_bwd", &gemm_fp8_swiglu_bwd);
    m.impl("gemm_fp8_rope", &gemm_fp8_rope);
    m.impl("cast_fp8", &cast_fp8);
    m.impl("transpose_bf16", &transpose_bf16);
    m.impl("cast_fp8_t", &cast_fp8_t);
    m.impl("swiglu_cast_fp8_t", &swiglu_cast_fp8_t);
    m.impl("add_rmsnorm_cast_fp8_t", &add_rmsnorm_cast_fp8_t);
    m.impl("update_scales", &update_scales);
    m.impl("masked_sdpa", &masked_sdpa);
    m.impl("softmax_fwd", &softmax_fwd);
    m.impl("softmax_bwd", &softmax_bwd);
    m.impl("rope", &rope);
    m.impl("fa_fwd", &fa_fwd);
    m.impl("fa_bwd", &fa_bwd);
    m.impl("rope_qk_", &rope_qk_);
    m.impl("kv_append", &kv_append);
    m.impl("decode_attn", &decode_attn);
    m.impl("decode_gemv", &decode_gemv);
    m.impl("decode_qkv", &decode_qkv);
    m.impl("decode_attn_proj", &decode_attn_proj);
}
