// Host-side launcher declarations for the gfx950 kernels.  Every launcher
// takes raw device pointers plus the HIP stream it must run on and never
// allocates or synchronises, so callers may capture it in a HIP graph.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

enum { DT_F32 = 0, DT_BF16 = 1 };

// rmsnorm.hip
void launch_rmsnorm_fwd(int dtype, const void* x, const void* w, void* y, float* rstd, int M, int N, float eps,
                        hipStream_t s);
void launch_add_rmsnorm_fwd(int dtype, const void* x, const void* d, const void* w, void* sum, void* y, float* rstd,
                            int M, int N, float eps, hipStream_t s);
int rmsnorm_bwd_grid(int M);
// dw_mode 0: dw = the column sums (activation dtype); 1 / 2: dw += them (a bf16 / fp32 gradient slot)
void launch_rmsnorm_bwd(int dtype, const void* dy, const void* x, const void* w, const float* rstd, void* dx,
                        float* partial, void* dw, const void* dres, int M, int N, hipStream_t s, int dw_mode = 0);

// activations.hip
void launch_swiglu_fwd(int dtype, const void* gu, void* out, size_t M, int F, hipStream_t s);
void launch_swiglu_bwd(int dtype, const void* dout, const void* gu, void* dgu, size_t M, int F, hipStream_t s);
void launch_act_fwd(int dtype, int kind, const void* x, void* y, size_t n, hipStream_t s);
void launch_act_bwd(int dtype, int kind, const void* dy, const void* x, void* dx, size_t n, hipStream_t s);

// cross_entropy.hip
void launch_ce_fwd_bwd(int dtype, void* logits, long ld, const int64_t* targets, float* loss, float* lse,
                       const float* nvalid, int M, int V, long ignore_index, int write_grad, hipStream_t s);

// embedding.hip
void launch_embed_fwd(int dtype, const void* W, const int64_t* ids, void* out, int M, int D, long vocab,
                      hipStream_t s);
void launch_embed_bwd(int dtype, const void* dout, const int64_t* sorted_ids, const int64_t* perm, void* dW, int M,
                      int D, hipStream_t s);

// optim.hip
void launch_adamw(int gdtype, float* p, float* m, float* v, const void* g, void* pout_bf16, size_t n, float lr,
                  double b1, double b2, float eps, float wd, float bc1, float bc2_sqrt, const float* gscale,
                  const int* nstep, const uint8_t* wd_mask, hipStream_t s);
void launch_adam_count(int* nstep, const float* gscale, hipStream_t s);
void launch_sumsq_partial(int dtype, const void* x, size_t n, float* partial, int nblocks, hipStream_t s);
void launch_norm_finalize(const float* partial, int np, float max_norm, float* out_norm, float* out_coef,
                          hipStream_t s);
void launch_scale(int dtype, void* x, size_t n, const float* coef, hipStream_t s);

// softmax.hip
// masked_sdpa.hip: the generic masked SDPA contract path (dtype: DT_F32 / DT_BF16; mask uint8, strides in bytes per
// (batch-head, query, key), null = no mask)
void launch_masked_sdpa(int dtype, const void* q, const void* k, const void* v, const uint8_t* mask, long msb,
                        long msq, long msk, void* o, int BH, int Sq, int Sk, int D, int Dv, float scale,
                        hipStream_t s);
void launch_softmax_fwd(int dtype, const void* x, void* y, int M, int N, hipStream_t s);
void launch_softmax_bwd(int dtype, const void* dy, const void* y, void* dx, int M, int N, hipStream_t s);

// fp8.hip
void launch_cast_fp8(int dtype, int fmt, const void* x, size_t n, const float* scale, void* out,
                     unsigned* amax_bits, hipStream_t s);  // fmt 0 = e4m3fn, 1 = e5m2
// dst[C, R] = src[R, C]^T, bf16, R and C multiples of 64 (16-byte aligned rows)
void launch_transpose_bf16(const void* src, long ld_src, void* dst, long ld_dst, int R, int C, hipStream_t s,
                           const float* scale = nullptr);
void launch_cast_fp8_t(const void* w, int N, int K, const float* scale, void* w8, void* w8t, unsigned* amax_bits,
                       int fmt, hipStream_t s);
// SwiGLU + two-layout fp8 cast (fp8.hip): mode 0 a = silu(g) u -> a8 [M][F], a8t [F][M] (e4m3); mode 1 the gate
// gradient from dout [M][F] -> dgu8 [M][2F], dgu8t [2F][M] (e5m2); gu = [g | u] [M][2F]; M, F multiples of 64
void launch_swiglu_cast_fp8_t(int mode, const void* gu, const void* dout, int M, int F, const float* scale, void* o8,
                              void* o8t, unsigned* amax_bits, hipStream_t s);
// residual add + RMSNorm written only as e4m3 in both layouts (fp8.hip): sum = x + d (bf16; d == nullptr: no add,
// nothing stored), rstd, y8 [M][N] and y8t [N][M]; bf16, M and N multiples of 128, N <= 2048
void launch_add_rmsnorm_cast_fp8_t(const void* x, const void* d, const void* w, void* sum, void* y8, void* y8t,
                                   float* rstd, int M, int N, float eps, const float* scale, unsigned* amax_bits,
                                   hipStream_t s);  // bf16 W [N][K] -> e4m3 w8 [N][K] and w8t [K][N]
void launch_update_scales(unsigned* amax_cur, float* hist, float* scale, float* inv_scale, int n, int H, int pos,
                          float margin, int fmt, hipStream_t s);

// gemm.hip.  C is bf16, or fp32 with c_f32 (gradient buffers); slab = fp32 partials [splits][Mo][No], required
// for splits > 1 or an fp32 C, null otherwise (one split written straight into the bf16 C)
size_t gemm_lds_bytes();
bool gemm_shape_ok(int Mo, int No, int R, int splits, int tile);
void launch_gemm(int a_kmajor, int b_kmajor, const void* A, long lda, const void* B, long ldb, void* C, long ldc,
                 float beta, int Mo, int No, int R, int splits, float* slab, int tile, int c_f32, hipStream_t s);

void splitk_reduce(const float* slab, void* C, long ldc, float beta, int M, int N, int splits, int c_f32,
                   hipStream_t s);

// gemm_pp.hip (8-wave ping-pong, 256 x 256 x 64 tiles, any operand layout); C / slab as launch_gemm
bool gemm_pp_shape_ok(int M, int N, int R, int splits);
void launch_gemm_pp(int a_kmajor, int b_kmajor, const void* A, long lda, const void* B, long ldb, void* C, long ldc,
                    float beta, int M, int N, int R, int splits, float* slab, int c_f32, hipStream_t s);

// grouped weight gradients: np <= 4 problems C_p (+)= dY_p^T X_p over the same R tokens in one split-K launch and
// one ordered reduce (X_p token-major, or X_p^T [N_p][R] with b_kmajor); slab: splits * sum M_p N_p floats
void launch_gemm_pp_dw_group(int np, const void* const* A, const long* lda, const void* const* B, const long* ldb,
                             int b_kmajor, void* const* C, const long* ldc, const int* M, const int* N, int R,
                             int splits, float beta, float* slab, int c_f32, hipStream_t s);

// fp8 x fp8 -> bf16 on the ping-pong kernel with v_mfma_scale_f32_16x16x128_f8f6f4: C = A8 B8^T * sa * sb,
// A8 [M][K] (fmt_a 0 e4m3 / 1 e5m2), B8 [N][K] e4m3, both K-major; strides in bytes (A, B) / elements (C)
// gu = (X8 . W13_8^T) * sa * sb with a = silu(g) u cast to e4m3 in both layouts + amax (fused fp8 SwiGLU forward)
void launch_gemm_fp8_swiglu(const void* A8, long lda, const void* B8, long ldb, void* gu, long ldg, void* a8,
                            void* a8t, int M, int F, int K, const float* sa, const float* sb, const float* a_scale,
                            unsigned* a_amax, hipStream_t s);
// da = G8 . W2t_8^T with the SwiGLU backward and the two-layout e5m2 cast of [dg | du] + amax (fused fp8 backward)
void launch_gemm_fp8_swiglu_bwd(const void* G8, long ldg8, const void* W8, long ldw8, const void* gu, void* dgu8,
                                void* dgu8t, int M, int F, int K, const float* sa, const float* sb,
                                const float* d_scale, unsigned* d_amax, hipStream_t s);
void launch_gemm_fp8(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                     int fmt_a, const float* sa, const float* sb, hipStream_t s);

void launch_gemm_pp_swiglu_fwd(const void* X, long ldx, const void* W13, long ldw, void* gu, long ldg, void* act,
                               long lda_, int M, int F, int R, hipStream_t s);
void launch_gemm_pp_swiglu_bwd(const void* dY, long ldy, const void* W2, long ldw, const void* gu, void* dgu,
                               long ldg, int M, int F, int R, hipStream_t s);

// rope.hip
void launch_rope_qk(void* qkv, long ld, const float* cosT, const float* sinT, long rows, int S, int H, int Hkv, int D,
                    hipStream_t s);
void launch_rope(int dtype, const void* x, void* y, const int64_t* pos, const float* cosT, const float* sinT,
                 size_t R, int H, int D, int inverse, hipStream_t s);

// flash_attn.hip
struct FaArgs {
    const __bf16* q;
    const __bf16* k;
    const __bf16* v;
    long ld_q, ld_kv;  // elements between consecutive tokens
    __bf16* o;         // [B, S, H, D] with row stride ld_o
    long ld_o;
    float* lse;        // [B, H, S] base-2 log-sum-exp of the scaled scores
    const float* cos;  // [S_max, D/2]
    const float* sin;
    int B, H, Hkv, S, D;
    int causal, rope;  // rope: 0 none, 1 fused (rotate Q/K on load, un-rotate dQ/dK), 2 Q/K pre-rotated (rope_qk_)
    float scale;
    // backward only
    const __bf16* dout;
    long ld_do;
    float* delta;   // [B, H, S] scratch
    float* dq_acc;  // [B, Spad, H, D] fp32 scratch (forward: zeroed there when non-null)
    int dq_zeroed;  // backward: dq_acc arrives zeroed (by the forward), the pre-kernel skips it
    __bf16* dq;
    long ld_dq;
    __bf16* dk;
    __bf16* dv;
    long ld_dkv;
    float* dkv_part;  // GQA only: [B*S][H][2][D] fp32 per-query-head dK / dV partials
};
// decode_attn.hip (KV-cache serving path; `pos` = device int32 position of the first new token)
int decode_attn_splits(int Lmax);
bool decode_attn_ok(int H, int Hkv, int D, int T);
void launch_decode_attn(const void* q, const void* k, const void* v, float* part, void* out, const int* pos, int B,
                        int T, int H, int Hkv, int D, int Lmax, float scale, hipStream_t s);
void launch_kv_append(const void* qkv, long ld, void* qo, void* Kc, void* Vc, const float* cosT, const float* sinT,
                      const int* pos, int B, int T, int H, int Hkv, int D, int Lmax, hipStream_t s);

// decode_gemv.hip (M <= 16 token rows; epi 0 plain, 1 SwiGLU over [W1; W3], 2 fused QKV + RoPE + KV-cache write)
struct GemvArgs {
    const __bf16* x;   // input rows [M][K] (row stride ldx)
    const __bf16* xd;  // optional delta added to x before the norm (residual add), same layout
    long ldx;
    const __bf16* ln;  // optional RMSNorm weight [K]
    float eps;
    __bf16* xsum;      // optional: x + xd written here [M][K] (workgroup 0)
    const __bf16* W;   // weight [N][K] (row stride ldw)
    long ldw;
    int N, K, M;
    __bf16* y;         // output [M][N] (epi 1: [M][N/2]; epi 2: q part [M][H*D]), row stride ldy
    long ldy;
    int H, Hkv, D, Lmax;  // epi 2 only
    const float* cosT;
    const float* sinT;
    const int* pos;
    __bf16* kc;
    __bf16* vc;
    const float* part;  // optional prologue: x = merged decode-attention partials [M][H][nsplit][D + 2] (H, D)
    int nsplit;
};
size_t gemv_lds_bytes(int M, int K);
bool gemv_ok(int M, int K);
void launch_gemv(const GemvArgs& a, int epi, hipStream_t s);

size_t fa_fwd_lds_bytes(int D);
size_t fa_bwd_lds_bytes(int D);
void launch_fa_fwd(const FaArgs& a, hipStream_t s);
// flash_attn_fwd_v4.hip: the D = 64 forward without in-kernel RoPE; false when not applicable / not selected
bool launch_fa_fwd_v4(const FaArgs& a, hipStream_t s);
int fa_fwd_config(int ver);  // the D = 64 forward: 8 (default) or 2 (fa_fwd_kernel); ver <= 0 leaves it unchanged;
                             // returns the version in force before the call
void launch_fa_bwd(const FaArgs& a, hipStream_t s);
// true when launch_fa_bwd takes the split form for head dim D and FaArgs::rope mode (no fp32 dQ accumulator, no pre
// / convert passes): D = 64 always, D = 128 unless rope == 1 (the in-kernel rotation; fa_bwd pre-rotates a copy)
bool fa_bwd_split_active(int D, int rope = 0);
// backward form 0 split / 1 fused; negative = unchanged; returns the form in force before the call
int fa_bwd_config(int mode);
// flash_attn_bwd_dq16.hip: the split backward's dQ kernel with 16 queries per wave (D = 64, rope 0 / 2) when
// fa_dq_config selected it; false when not applicable / not selected.  fa_dq_config: 0 = 32 queries per wave, 1 = 16
// (8 waves), 2 = 16 (4 waves), 3 = 1 up to S = 2048 else 0 (default); negative = unchanged; returns the previous form
bool launch_fa_bwd_dq16(const FaArgs& a, hipStream_t s);
bool fa_read_stamps_dq16(long long* host, int n);
int fa_dq_config(int form);
// per-workgroup s_memtime stamps of the last split-backward launch (BPE_FA_STAMPS builds only; false otherwise)
bool fa_read_stamps(long long* host, int n);
// per-workgroup s_memtime stamps of the last gemm_pp launch (BPE_GPP_STAMPS builds only; false otherwise)
bool gpp_read_stamps(long long* host, int n);
// per-wave phase stamps of the last one-tile gemm_pp launch (BPE_GPP_PHASE_STAMPS builds only; false otherwise)
bool gpp_read_phase_stamps(long long* host, int n);
// gemm_pp: 1 = persistent kernel for the one-pass bf16 / fp8 GEMMs, 0 = one tile per workgroup; -1 queries.
// Returns the previous mode.
int gpp_persist_config(int mode);
// tile order of the one-pass ping-pong GEMMs: 0 = row-major, n > 0 = column-major in bands of n row blocks; -1 reads
int gpp_order_config(int gm);
// C = beta * C + (A8 . B8^T) * sa * sb over `splits` fp32 partials (slab [splits][M][N]); C bf16 or fp32 (c_f32)
void launch_gemm_fp8_splitk(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                            int fmt_a, const float* sa, const float* sb, float beta, int splits, float* slab,
                            int c_f32, hipStream_t s);
// qkv = X . Wqkv^T (bf16, both K-major) with RoPE applied to output columns [0, rot_cols) in the epilogue
void launch_gemm_pp_rope(const void* X, long ldx, const void* W, long ldw, void* C, long ldc, int M, int N, int R,
                         const float* cosT, const float* sinT, int S, int D, int rot_cols, hipStream_t s);
// the fp8 (e4m3 x e4m3) QKV projection with RoPE on output columns [0, rot_cols) in the epilogue (strides in bytes
// for A / B)
void launch_gemm_fp8_rope(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                          const float* sa, const float* sb, const float* cosT, const float* sinT, int S, int D,
                          int rot_cols, hipStream_t s);
// whether FaArgs::dkv_part (GQA fp32 dK / dV partials of the fused backward) must be set
bool fa_dkv_partials_needed(int D, int rope = 0);
