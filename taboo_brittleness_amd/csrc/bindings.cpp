// PyTorch bindings for the gfx950 kernels (module `_tb_kernels`).
//
// Every op is "out=" style: the Python runtime preallocates its workspaces once
// so the decode step can be captured into a hipGraph without allocations
// (cdna_hip_programming.md Guideline 9).  All launches go to the current HIP
// stream of the calling thread.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>

#include <cstdlib>

#include "api.h"

namespace {

// PyTorch-ROCm exposes HIP devices as "cuda"; the masquerading stream is the
// stream torch itself launches on (and captures into hipGraphs).
hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bfloat16")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define CHECK_I32(t) TORCH_CHECK((t).scalar_type() == at::kInt, #t " must be int32")
#define CHECK_U8(t) TORCH_CHECK((t).scalar_type() == at::kByte || (t).scalar_type() == at::kBool, #t " must be uint8/bool")
#define IN_BF16(t) CHECK_DEV(t); CHECK_CONTIG(t); CHECK_BF16(t)
#define IN_F32(t) CHECK_DEV(t); CHECK_CONTIG(t); CHECK_F32(t)
#define IN_I32(t) CHECK_DEV(t); CHECK_CONTIG(t); CHECK_I32(t)
#define IN_U8(t) CHECK_DEV(t); CHECK_CONTIG(t); CHECK_U8(t)

// TB_DEBUG_CHECKS=1: extra device-syncing argument checks (index ranges); never inside a stream capture.
bool debug_checks() {
  static const bool on = [] {
    const char* e = std::getenv("TB_DEBUG_CHECKS");
    return e != nullptr && e[0] == '1';
  }();
  if (!on) return false;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(cur_stream(), &st) != hipSuccess) return false;
  return st == hipStreamCaptureStatusNone;
}

inline uint16_t* bf(torch::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }
inline const uint16_t* cbf(const torch::Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
inline const float* optf(const c10::optional<torch::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->is_cuda(), "optional f32 tensor");
  return t->data_ptr<float>();
}

void rmsnorm(torch::Tensor x, torch::Tensor w, torch::Tensor y, double eps) {
  IN_BF16(x); IN_BF16(w); IN_BF16(y);
  const int D = x.size(-1), M = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && w.numel() == D && y.numel() == x.numel(), "rmsnorm shapes");
  c10::DeviceGuard g(x.device());
  tb_rmsnorm(cbf(x), cbf(w), bf(y), M, D, (float)eps, cur_stream());
}

void add_rmsnorm2(torch::Tensor h, torch::Tensor o, torch::Tensor w_post, torch::Tensor w_next, torch::Tensor x,
                  double eps) {
  IN_BF16(h); IN_BF16(o); IN_BF16(w_post); IN_BF16(w_next); IN_BF16(x);
  const int D = h.size(-1), M = h.numel() / D;
  TORCH_CHECK(D % 8 == 0 && o.numel() == h.numel() && x.numel() == h.numel(), "add_rmsnorm2 shapes");
  c10::DeviceGuard g(h.device());
  tb_add_rmsnorm2(bf(h), cbf(o), cbf(w_post), cbf(w_next), bf(x), M, D, (float)eps, cur_stream());
}

// add_rmsnorm2 with o given as ks fp32 split-K partials [ks, M, D] (gemm4_splitk_part)
void add_rmsnorm2_part(torch::Tensor h, torch::Tensor part, int64_t ks, torch::Tensor w_post, torch::Tensor w_next,
                       torch::Tensor x, double eps) {
  IN_BF16(h); IN_F32(part); IN_BF16(w_post); IN_BF16(w_next); IN_BF16(x);
  const int D = h.size(-1), M = h.numel() / D;
  TORCH_CHECK(D % 8 == 0 && x.numel() == h.numel() && ks >= 1 && part.numel() >= ks * (int64_t)M * D,
              "add_rmsnorm2_part shapes");
  c10::DeviceGuard g(h.device());
  tb_add_rmsnorm2_part(bf(h), part.data_ptr<float>(), (int)ks, cbf(w_post), cbf(w_next), bf(x), M, D, (float)eps,
                       cur_stream());
}

void embed_rmsnorm(torch::Tensor ids, torch::Tensor E, torch::Tensor w, torch::Tensor h, torch::Tensor x,
                   double scale, double eps) {
  IN_I32(ids); IN_BF16(E); IN_BF16(w); IN_BF16(h); IN_BF16(x);
  const int D = E.size(1), V = E.size(0), M = ids.numel();
  TORCH_CHECK(D % 8 == 0 && h.numel() == (int64_t)M * D && x.numel() == h.numel(), "embed shapes");
  c10::DeviceGuard g(E.device());
  tb_embed_rmsnorm(ids.data_ptr<int32_t>(), cbf(E), cbf(w), bf(h), bf(x), M, D, V, (float)scale, (float)eps,
                   cur_stream());
}

void rope_qkv_cache(torch::Tensor qkv, torch::Tensor pos, torch::Tensor slot_of_row, torch::Tensor cos_t,
                    torch::Tensor sin_t, torch::Tensor q_out, torch::Tensor kc, torch::Tensor vc, int64_t Hq,
                    int64_t Hkv, int64_t HD) {
  IN_BF16(qkv); IN_I32(pos); IN_I32(slot_of_row); IN_F32(cos_t); IN_F32(sin_t); IN_BF16(q_out); IN_BF16(kc);
  IN_BF16(vc);
  const int M = pos.numel();
  TORCH_CHECK(qkv.numel() == (int64_t)M * (Hq + 2 * Hkv) * HD, "qkv shape");
  TORCH_CHECK(q_out.numel() == (int64_t)M * Hq * HD, "q_out shape");
  TORCH_CHECK(kc.dim() == 4 && kc.size(1) == Hkv && kc.size(3) == HD && vc.sizes() == kc.sizes(), "cache shape");
  TORCH_CHECK(cos_t.size(1) == HD / 2 && sin_t.sizes() == cos_t.sizes(), "rope table shape");
  TORCH_CHECK(HD % 16 == 0, "head_dim must be a multiple of 16");
  c10::DeviceGuard g(qkv.device());
  tb_rope_qkv_cache(cbf(qkv), pos.data_ptr<int32_t>(), slot_of_row.data_ptr<int32_t>(), cos_t.data_ptr<float>(),
                    sin_t.data_ptr<float>(), bf(q_out), bf(kc), bf(vc), M, Hq, Hkv, HD, kc.size(2), cos_t.size(0),
                    cur_stream());
}

// rope_qkv_cache from the QKV projection's ks fp32 split-K partials (gemm4_splitk_part) instead of its bf16 output
void rope_qkv_cache_part(torch::Tensor part, int64_t ks, torch::Tensor pos, torch::Tensor slot_of_row,
                         torch::Tensor cos_t, torch::Tensor sin_t, torch::Tensor q_out, torch::Tensor kc, torch::Tensor vc,
                         int64_t Hq, int64_t Hkv, int64_t HD) {
  IN_F32(part); IN_I32(pos); IN_I32(slot_of_row); IN_F32(cos_t); IN_F32(sin_t); IN_BF16(q_out); IN_BF16(kc);
  IN_BF16(vc);
  const int M = pos.numel();
  TORCH_CHECK(ks >= 1 && part.numel() >= ks * (int64_t)M * (Hq + 2 * Hkv) * HD, "partials shape");
  TORCH_CHECK(q_out.numel() == (int64_t)M * Hq * HD, "q_out shape");
  TORCH_CHECK(kc.dim() == 4 && kc.size(1) == Hkv && kc.size(3) == HD && vc.sizes() == kc.sizes(), "cache shape");
  TORCH_CHECK(cos_t.size(1) == HD / 2 && sin_t.sizes() == cos_t.sizes(), "rope table shape");
  TORCH_CHECK(HD % 16 == 0, "head_dim must be a multiple of 16");
  c10::DeviceGuard g(part.device());
  tb_rope_qkv_cache_part(part.data_ptr<float>(), (int)ks, pos.data_ptr<int32_t>(), slot_of_row.data_ptr<int32_t>(),
                         cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), bf(q_out), bf(kc), bf(vc), M, Hq, Hkv, HD,
                         kc.size(2), cos_t.size(0), cur_stream());
}

void kv_fanout(torch::Tensor kc, torch::Tensor vc, torch::Tensor src_row, torch::Tensor slot, torch::Tensor pos,
               int64_t nlayers) {
  IN_BF16(kc); IN_BF16(vc); IN_I32(src_row); IN_I32(slot); IN_I32(pos);
  TORCH_CHECK(kc.dim() == 5 && vc.sizes() == kc.sizes(), "kv_fanout: caches must be [L, slots, Hkv, S, HD]");
  TORCH_CHECK(nlayers >= 0 && nlayers <= kc.size(0), "kv_fanout: nlayers out of range");
  TORCH_CHECK(kc.size(4) % 8 == 0, "kv_fanout: head_dim must be a multiple of 8");
  const int M = src_row.numel();
  TORCH_CHECK(slot.numel() >= M && pos.numel() >= M, "kv_fanout: slot/pos shorter than src_row");
  if (debug_checks() && M > 0) {
    const auto sl = slot.narrow(0, 0, M);
    TORCH_CHECK(sl.min().item<int>() >= 0 && sl.max().item<int>() < kc.size(1), "kv_fanout: slot out of range");
    TORCH_CHECK(src_row.max().item<int>() < M, "kv_fanout: src_row out of range");
  }
  c10::DeviceGuard g(kc.device());
  tb_kv_fanout(bf(kc), bf(vc), src_row.data_ptr<int32_t>(), slot.data_ptr<int32_t>(), pos.data_ptr<int32_t>(), M,
               (int)nlayers, kc.size(1), kc.size(2), kc.size(3), kc.size(4), cur_stream());
}

void attention(torch::Tensor q, torch::Tensor kc, torch::Tensor vc, torch::Tensor out, torch::Tensor pos,
               torch::Tensor slot, int64_t B, int64_t T, double scale, double softcap, int64_t window) {
  IN_BF16(q); IN_BF16(kc); IN_BF16(vc); IN_BF16(out); IN_I32(pos); IN_I32(slot);
  TORCH_CHECK(kc.dim() == 4, "cache must be [slots, Hkv, S, HD]");
  const int Hkv = kc.size(1), S = kc.size(2), HD = kc.size(3);
  TORCH_CHECK(q.numel() % (B * T * HD) == 0, "q shape");
  const int Hq = q.numel() / (B * T * HD);
  TORCH_CHECK(Hq % Hkv == 0, "GQA ratio");
  const int G = Hq / Hkv;
  TORCH_CHECK((HD == 256 || HD == 128) && (G == 1 || G == 2 || G == 4), "unsupported head geometry");
  TORCH_CHECK(pos.numel() == B * T && slot.numel() >= B && out.numel() == q.numel(), "attention shapes");
  c10::DeviceGuard g(q.device());
  tb_attention(cbf(q), cbf(kc), cbf(vc), bf(out), pos.data_ptr<int32_t>(), slot.data_ptr<int32_t>(), B, T, Hq, Hkv,
               HD, S, (float)scale, (float)softcap, (int)window, cur_stream());
}

void attention_prefix(torch::Tensor q, torch::Tensor kc, torch::Tensor vc, torch::Tensor out, torch::Tensor pos,
                      torch::Tensor slot, int64_t B, double scale, double softcap, int64_t window, torch::Tensor pk,
                      torch::Tensor pv, torch::Tensor pslot, torch::Tensor plen) {
  IN_BF16(q); IN_BF16(kc); IN_BF16(vc); IN_BF16(out); IN_I32(pos); IN_I32(slot);
  IN_BF16(pk); IN_BF16(pv); IN_I32(pslot); IN_I32(plen);
  TORCH_CHECK(kc.dim() == 4, "cache must be [slots, Hkv, S, HD]");
  const int Hkv = kc.size(1), S = kc.size(2), HD = kc.size(3);
  TORCH_CHECK(S <= 8192, "shared-prefix attention is the decode kernel (S <= 8192)");
  TORCH_CHECK(q.numel() % (B * HD) == 0, "q shape");
  const int Hq = q.numel() / (B * HD);
  TORCH_CHECK(Hq % Hkv == 0, "GQA ratio");
  const int G = Hq / Hkv;
  TORCH_CHECK((HD == 256 || HD == 128) && (G == 1 || G == 2 || G == 4), "unsupported head geometry");
  TORCH_CHECK(pos.numel() == B && slot.numel() >= B && out.numel() == q.numel(), "attention shapes (T == 1)");
  TORCH_CHECK(pk.dim() == 4 && pk.size(1) == Hkv && pk.size(2) == S && pk.size(3) == HD && pv.sizes() == pk.sizes(),
              "prefix cache must be [P, Hkv, S, HD] like the cache");
  TORCH_CHECK(pslot.numel() >= B && plen.numel() >= B, "prefix slot/len per row");
  c10::DeviceGuard g(q.device());
  tb_attention(cbf(q), cbf(kc), cbf(vc), bf(out), pos.data_ptr<int32_t>(), slot.data_ptr<int32_t>(), B, 1, Hq, Hkv,
               HD, S, (float)scale, (float)softcap, (int)window, cur_stream(), cbf(pk), cbf(pv),
               pslot.data_ptr<int32_t>(), plen.data_ptr<int32_t>());
}

void attention_varlen(torch::Tensor q, torch::Tensor kc, torch::Tensor vc, torch::Tensor out, torch::Tensor pos,
                      torch::Tensor blk, double scale, double softcap, int64_t window) {
  IN_BF16(q); IN_BF16(kc); IN_BF16(vc); IN_BF16(out); IN_I32(pos); IN_I32(blk);
  TORCH_CHECK(kc.dim() == 4, "cache must be [slots, Hkv, S, HD]");
  const int Hkv = kc.size(1), S = kc.size(2), HD = kc.size(3);
  const int M = pos.numel();
  TORCH_CHECK(q.numel() % ((int64_t)M * HD) == 0 && out.numel() == q.numel(), "q/out shape");
  const int Hq = q.numel() / ((int64_t)M * HD);
  TORCH_CHECK(Hq % Hkv == 0 && (HD == 256 || HD == 128), "unsupported head geometry");
  const int G = Hq / Hkv;
  TORCH_CHECK(G == 1 || G == 2 || G == 4, "unsupported GQA ratio");
  TORCH_CHECK(blk.dim() == 2 && blk.size(1) == 3, "blk must be [nblk, 3] = (row0, nrows, slot)");
  c10::DeviceGuard g(q.device());
  tb_attention_varlen(cbf(q), cbf(kc), cbf(vc), bf(out), pos.data_ptr<int32_t>(), blk.data_ptr<int32_t>(),
                      blk.size(0), Hq, Hkv, HD, S, (float)scale, (float)softcap, (int)window, cur_stream());
}

// Varlen attention whose blocks read keys [0, plen) from a shared prefix cache slot:
// blk [nblk, 5] = (row0, nrows, slot, prefix slot, prefix length).
void attention_varlen_prefix(torch::Tensor q, torch::Tensor kc, torch::Tensor vc, torch::Tensor out, torch::Tensor pos,
                             torch::Tensor blk, double scale, double softcap, int64_t window, torch::Tensor pk,
                             torch::Tensor pv) {
  IN_BF16(q); IN_BF16(kc); IN_BF16(vc); IN_BF16(out); IN_I32(pos); IN_I32(blk); IN_BF16(pk); IN_BF16(pv);
  TORCH_CHECK(kc.dim() == 4, "cache must be [slots, Hkv, S, HD]");
  const int Hkv = kc.size(1), S = kc.size(2), HD = kc.size(3);
  const int M = pos.numel();
  TORCH_CHECK(q.numel() % ((int64_t)M * HD) == 0 && out.numel() == q.numel(), "q/out shape");
  const int Hq = q.numel() / ((int64_t)M * HD);
  TORCH_CHECK(Hq % Hkv == 0 && (HD == 256 || HD == 128), "unsupported head geometry");
  const int G = Hq / Hkv;
  TORCH_CHECK(G == 1 || G == 2 || G == 4, "unsupported GQA ratio");
  TORCH_CHECK(blk.dim() == 2 && blk.size(1) == 5, "blk must be [nblk, 5] = (row0, nrows, slot, pslot, plen)");
  TORCH_CHECK(pk.dim() == 4 && pk.size(1) == Hkv && pk.size(2) == S && pk.size(3) == HD && pv.sizes() == pk.sizes(),
              "prefix cache must be [P, Hkv, S, HD] like the cache");
  c10::DeviceGuard g(q.device());
  tb_attention_varlen(cbf(q), cbf(kc), cbf(vc), bf(out), pos.data_ptr<int32_t>(), blk.data_ptr<int32_t>(),
                      blk.size(0), Hq, Hkv, HD, S, (float)scale, (float)softcap, (int)window, cur_stream(), 5,
                      cbf(pk), cbf(pv));
}

void geglu(torch::Tensor gu, torch::Tensor out) {
  IN_BF16(gu); IN_BF16(out);
  const int F2 = gu.size(-1), M = gu.numel() / F2;
  TORCH_CHECK(F2 % 16 == 0 && out.numel() == (int64_t)M * (F2 / 2), "geglu shapes");
  c10::DeviceGuard g(gu.device());
  tb_geglu(cbf(gu), bf(out), M, F2 / 2, cur_stream());
}

void argmax_rows(torch::Tensor logits, torch::Tensor out, double cap) {
  IN_BF16(logits); IN_I32(out);
  const int V = logits.size(-1), R = logits.numel() / V;
  TORCH_CHECK(out.numel() == R, "argmax out");
  c10::DeviceGuard g(logits.device());
  tb_argmax_rows(cbf(logits), out.data_ptr<int32_t>(), R, V, (float)cap, cur_stream());
}

void row_lse(torch::Tensor logits, torch::Tensor lse, double cap, bool emulate_bf16) {
  IN_BF16(logits); IN_F32(lse);
  const int V = logits.size(-1), R = logits.numel() / V;
  TORCH_CHECK(lse.numel() == R, "lse out");
  c10::DeviceGuard g(logits.device());
  tb_row_lse(cbf(logits), lse.data_ptr<float>(), R, V, (float)cap, emulate_bf16 ? 1 : 0, cur_stream());
}

// rowmap (optional, int32 [R_logical]): logical row r reads logits / lse row rowmap[r] (deduplicated rows).
const int32_t* rowmap_ptr(const c10::optional<torch::Tensor>& rowmap, int64_t R_phys, int64_t R_log) {
  if (!rowmap.has_value()) return nullptr;
  IN_I32((*rowmap));
  TORCH_CHECK(rowmap->numel() == R_log, "rowmap must have one entry per logical row");
  if (debug_checks() && R_log > 0)
    TORCH_CHECK(rowmap->min().item<int>() >= 0 && rowmap->max().item<int>() < R_phys, "rowmap out of range");
  return rowmap->data_ptr<int32_t>();
}

void gather_probs(torch::Tensor logits, torch::Tensor lse, torch::Tensor ids, torch::Tensor out, bool round_bf16,
                  c10::optional<torch::Tensor> rowmap) {
  IN_BF16(logits); IN_F32(lse); IN_I32(ids); IN_F32(out);
  const int V = logits.size(-1);
  const int Rp = logits.numel() / V;
  const int R = rowmap.has_value() ? rowmap->numel() : Rp;
  TORCH_CHECK(R > 0 ? (ids.numel() % R == 0 && out.numel() == ids.numel()) : ids.numel() == 0, "gather shapes");
  TORCH_CHECK(lse.numel() == Rp, "gather_probs: lse must have one entry per logits row");
  const int K = R > 0 ? ids.numel() / R : 0;
  const int32_t* rm = rowmap_ptr(rowmap, Rp, R);
  c10::DeviceGuard g(logits.device());
  tb_gather_probs(cbf(logits), lse.data_ptr<float>(), ids.data_ptr<int32_t>(), out.data_ptr<float>(), R, K, V,
                  round_bf16 ? 1 : 0, rm, cur_stream());
}

void lens_colsum(torch::Tensor logits, torch::Tensor lse, c10::optional<torch::Tensor> mask, torch::Tensor excl,
                 torch::Tensor acc, int64_t B, int64_t T, bool accumulate, bool round_bf16,
                 c10::optional<torch::Tensor> offs, c10::optional<torch::Tensor> cum,
                 c10::optional<torch::Tensor> rowmap) {
  IN_BF16(logits); IN_F32(lse); IN_I32(excl); IN_F32(acc);
  const int V = logits.size(-1);
  const int64_t Rp = logits.numel() / V;
  const int64_t R = rowmap.has_value() ? rowmap->numel() : Rp;      // logical rows (excl, mask, offs)
  TORCH_CHECK(lse.numel() == Rp && excl.numel() == 2 * R && acc.numel() == B * V, "lens_colsum shapes");
  const int32_t* rm = rowmap_ptr(rowmap, Rp, R);
  TORCH_CHECK(rm == nullptr || offs.has_value(), "lens_colsum rowmap is packed-layout only");
  const uint8_t* mp = nullptr;
  if (mask.has_value()) {
    IN_U8((*mask));
    TORCH_CHECK(mask->numel() == R, "lens_colsum mask");
    mp = reinterpret_cast<const uint8_t*>(mask->data_ptr());
  }
  const int32_t* op = nullptr;
  if (offs.has_value()) {
    IN_I32((*offs));
    TORCH_CHECK(offs->numel() == B + 1, "lens_colsum offs must be [B+1]");
    op = offs->data_ptr<int32_t>();
    TORCH_CHECK(!cum.has_value(), "cum is dense-layout only");
  } else {
    TORCH_CHECK(R == B * T, "lens_colsum dense layout needs B*T rows");
  }
  float* cp = nullptr;
  if (cum.has_value()) {
    IN_F32((*cum));
    TORCH_CHECK(cum->numel() == B * (T + 1) * V, "lens_colsum cum must be [B, T+1, V]");
    cp = cum->data_ptr<float>();
  }
  c10::DeviceGuard g(logits.device());
  tb_lens_colsum(cbf(logits), lse.data_ptr<float>(), mp, excl.data_ptr<int32_t>(), acc.data_ptr<float>(), B, T, V,
                 accumulate ? 1 : 0, round_bf16 ? 1 : 0, op, cp, rm, cur_stream());
}

void topk_rows(torch::Tensor x, torch::Tensor vals, torch::Tensor idx, int64_t K) {
  IN_F32(x); IN_F32(vals); IN_I32(idx);
  const int V = x.size(-1), R = x.numel() / V;
  TORCH_CHECK(K >= 1 && K <= 64 && K <= V && vals.numel() == R * K && idx.numel() == R * K, "topk shapes");
  c10::DeviceGuard g(x.device());
  const int C = tb_topk_chunks(R, V);
  torch::Tensor wv, wi;
  if (C > 1) {
    wv = torch::empty({(int64_t)R * C * K}, x.options());
    wi = torch::empty({(int64_t)R * C * K}, idx.options());
  }
  tb_topk_rows(x.data_ptr<float>(), vals.data_ptr<float>(), idx.data_ptr<int32_t>(), R, V, K,
               C > 1 ? wv.data_ptr<float>() : nullptr, C > 1 ? wi.data_ptr<int32_t>() : nullptr, C, cur_stream());
}

void xent_rows(torch::Tensor logits, torch::Tensor tgt, torch::Tensor nll, double cap, bool emulate_bf16) {
  IN_BF16(logits); IN_I32(tgt); IN_F32(nll);
  const int V = logits.size(-1), R = logits.numel() / V;
  TORCH_CHECK(tgt.numel() == R && nll.numel() == R, "xent shapes");
  c10::DeviceGuard g(logits.device());
  tb_xent_rows(cbf(logits), tgt.data_ptr<int32_t>(), nll.data_ptr<float>(), R, V, (float)cap, emulate_bf16 ? 1 : 0,
               cur_stream());
}

void register_softcap_table(torch::Tensor tab, double cap) {
  CHECK_DEV(tab); CHECK_CONTIG(tab);
  TORCH_CHECK(tab.scalar_type() == at::kBFloat16 && tab.numel() == 32768, "softcap table: 32768 bf16 entries");
  c10::DeviceGuard g(tab.device());
  tb_register_softcap_table((float)cap, reinterpret_cast<const uint16_t*>(tab.data_ptr()));
}

// Compact exact softcap (lens.hip CapC): tab = the reference table's entries [lo, hi) (bf16 magnitudes); |x| < lo is
// computed as rbf(rbf(x / cap) * cap), [hi, inf] saturates at sat — ops._softcap_table checks both exhaustively.
bool register_softcap_compact(torch::Tensor tab, double cap, int64_t lo, int64_t hi, double sat) {
  CHECK_DEV(tab); CHECK_CONTIG(tab);
  TORCH_CHECK(tab.scalar_type() == at::kBFloat16 && tab.numel() == hi - lo, "compact softcap table: hi - lo bf16 entries");
  c10::DeviceGuard g(tab.device());
  return tb_register_softcap_compact((float)cap, reinterpret_cast<const uint16_t*>(tab.data_ptr()), (int)lo, (int)hi,
                                     (float)sat);
}

// y[i] = exact bf16 softcap of x[i] (fp32 values) through the compact path; false if none is registered for cap
bool softcap_compact(torch::Tensor x, torch::Tensor y, double cap) {
  IN_BF16(x); IN_F32(y);
  TORCH_CHECK(y.numel() == x.numel(), "softcap_compact: shapes");
  c10::DeviceGuard g(x.device());
  return tb_softcap_compact(cbf(x), y.data_ptr<float>(), (int)x.numel(), (float)cap, cur_stream());
}

void decode_head(torch::Tensor logits, c10::optional<torch::Tensor> tgt, torch::Tensor nxt, torch::Tensor nll_self,
                 c10::optional<torch::Tensor> nll_tgt, double cap) {
  IN_BF16(logits); IN_I32(nxt); IN_F32(nll_self);
  const int V = logits.size(-1), R = logits.numel() / V;
  TORCH_CHECK(nxt.numel() == R && nll_self.numel() == R, "decode_head shapes");
  TORCH_CHECK(tgt.has_value() == nll_tgt.has_value(), "decode_head: tgt and nll_tgt go together");
  const int32_t* tp = nullptr;
  float* np = nullptr;
  if (tgt.has_value()) {
    IN_I32((*tgt)); IN_F32((*nll_tgt));
    TORCH_CHECK(tgt->numel() == R && nll_tgt->numel() == R, "decode_head teacher shapes");
    tp = tgt->data_ptr<int32_t>();
    np = nll_tgt->data_ptr<float>();
  }
  c10::DeviceGuard g(logits.device());
  tb_decode_head(cbf(logits), tp, nxt.data_ptr<int32_t>(), nll_self.data_ptr<float>(), np, R, V, (float)cap,
                 cur_stream());
}

// vocab-parallel decode head (this rank's V columns of the logits): float4 stats per row for vp_head_merge; returns
// false (nothing launched) when the cap has no registered softcap table
bool decode_head_stats(torch::Tensor logits, c10::optional<torch::Tensor> tgt, int64_t off, torch::Tensor stats,
                       double cap) {
  IN_BF16(logits); IN_F32(stats);
  const int V = logits.size(-1), R = logits.numel() / V;
  TORCH_CHECK(stats.numel() == (int64_t)R * 4, "decode_head_stats: stats must hold R x 4 floats");
  const int32_t* tp = nullptr;
  if (tgt.has_value() && tgt->defined()) {
    IN_I32((*tgt));
    TORCH_CHECK(tgt->numel() == R, "decode_head_stats: tgt shape");
    tp = tgt->data_ptr<int32_t>();
  }
  c10::DeviceGuard g(logits.device());
  return tb_decode_head_stats(cbf(logits), tp, (int)off, stats.data_ptr<float>(), R, V, (float)cap, cur_stream());
}


void gemm_nt(torch::Tensor A, torch::Tensor W, torch::Tensor C, c10::optional<torch::Tensor> bias,
             c10::optional<torch::Tensor> thr, int64_t epi) {
  IN_BF16(A); IN_BF16(W); CHECK_DEV(C); CHECK_CONTIG(C);
  const int K = A.size(-1), M = A.numel() / K, N = W.size(0);
  TORCH_CHECK(W.size(1) == K && K % 32 == 0, "gemm_nt: K must match and be a multiple of 32");
  TORCH_CHECK(C.numel() == (int64_t)M * N, "gemm_nt: C shape");
  TORCH_CHECK(epi >= 0 && epi <= 2, "gemm_nt: epi must be 0, 1 or 2");
  if (epi == 2) {
    TORCH_CHECK(!bias.has_value() || !bias->defined() || bias->numel() == N, "gemm_nt: bias numel must be N");
    TORCH_CHECK(!thr.has_value() || !thr->defined() || thr->numel() == N, "gemm_nt: thr numel must be N");
  }
  if (epi == 0) {
    TORCH_CHECK(C.scalar_type() == at::kBFloat16, "epi 0 writes bf16");
  } else {
    TORCH_CHECK(C.scalar_type() == at::kFloat, "epi 1/2 write f32");
  }
  c10::DeviceGuard g(A.device());
  tb_gemm_nt(cbf(A), cbf(W), C.data_ptr(), optf(bias), optf(thr), M, N, K, N, (int)epi, cur_stream());
}

// Four-wave 256x256x64 (tile_rows = 128: 128x256x64) MFMA GEMM (gemm4.hip): the same epilogues, operand layouts
// and numerics as the ring GEMM (bit-identical outputs), 128x128 wave tiles.
void gemm4(torch::Tensor A, torch::Tensor W, torch::Tensor C, c10::optional<torch::Tensor> bias,
           c10::optional<torch::Tensor> thr, int64_t epi, int64_t tile_rows) {
  IN_BF16(A); IN_BF16(W); CHECK_DEV(C); CHECK_CONTIG(C);
  TORCH_CHECK(W.dim() == 2, "gemm4: W must be [N, K]");
  TORCH_CHECK(tile_rows == 256 || tile_rows == 128, "gemm4: tile_rows must be 256 or 128");
  const int K = A.size(-1), M = A.numel() / K, N = W.size(0);
  TORCH_CHECK(W.size(1) == K, "gemm4: K mismatch");
  TORCH_CHECK(tb_gemm4_ok(M, N, K), "gemm4: need N % 256 == 0, K % 64 == 0, K >= 64");
  TORCH_CHECK(epi >= 0 && epi <= 3, "gemm4: epi must be 0..3");
  const int64_t ncols = epi == 3 ? N / 2 : N;
  TORCH_CHECK(C.numel() == (int64_t)M * ncols, "gemm4: C shape");
  TORCH_CHECK(C.scalar_type() == ((epi == 0 || epi == 3) ? at::kBFloat16 : at::kFloat), "gemm4: C dtype");
  if (epi == 2) {
    TORCH_CHECK(!bias.has_value() || !bias->defined() || bias->numel() == N, "gemm4: bias numel must be N");
    TORCH_CHECK(!thr.has_value() || !thr->defined() || thr->numel() == N, "gemm4: thr numel must be N");
  }
  c10::DeviceGuard g(A.device());
  tb_gemm4(cbf(A), cbf(W), C.data_ptr(), epi == 2 ? optf(bias) : nullptr, epi == 2 ? optf(thr) : nullptr, M, N, K,
           (int)ncols, (int)epi, (int)tile_rows, cur_stream());
}

bool gemm4_ok(int64_t M, int64_t N, int64_t K) { return tb_gemm4_ok(M, N, K); }

// Ring GEMM (gemm_ring.hip): batch-invariant narrow tiles bm x bn for decode / mid row counts; epi 0 bf16 [M, N],
// epi 3 GeGLU of the interleaved gate|up rows (bf16 [M, N/2]).  Bit-identical to gemm4 at every M.
void gemm_ring(torch::Tensor A, torch::Tensor W, torch::Tensor C, int64_t epi, int64_t bm, int64_t bn, int64_t var) {
  IN_BF16(A); IN_BF16(W); IN_BF16(C);
  TORCH_CHECK(W.dim() == 2, "gemm_ring: W must be [N, K]");
  const int K = A.size(-1), M = A.numel() / K, N = W.size(0);
  TORCH_CHECK(W.size(1) == K, "gemm_ring: K mismatch");
  TORCH_CHECK(epi == 0 || epi == 3, "gemm_ring: epi must be 0 or 3");
  TORCH_CHECK(tb_gemm_ring_ok(M, N, K, (int)epi, (int)bm, (int)bn, (int)var), "gemm_ring: unsupported tile / shape");
  const int64_t ncols = epi == 3 ? N / 2 : N;
  TORCH_CHECK(C.numel() == (int64_t)M * ncols, "gemm_ring: C shape");
  c10::DeviceGuard g(A.device());
  tb_gemm_ring(cbf(A), cbf(W), bf(C), M, N, K, (int)ncols, (int)epi, (int)bm, (int)bn, (int)var, cur_stream());
}

bool gemm_ring_ok(int64_t M, int64_t N, int64_t K, int64_t epi, int64_t bm, int64_t bn, int64_t var) {
  return tb_gemm_ring_ok(M, N, K, (int)epi, (int)bm, (int)bn, (int)var);
}

std::vector<std::pair<int64_t, int64_t>> gemm_ring_tiles(int64_t epi) {
  int bm[64], bn[64];
  const int n = std::min(64, tb_gemm_ring_tiles((int)epi, bm, bn, 64));
  std::vector<std::pair<int64_t, int64_t>> out;
  for (int i = 0; i < n; ++i) out.emplace_back(bm[i], bn[i]);
  return out;
}

// QKV projection + RoPE + KV-cache scatter on the ring GEMM (gemm4_qkv_rope's epilogue, narrow tiles)
void gemm_ring_qkv_rope(torch::Tensor x, torch::Tensor w, torch::Tensor pos, torch::Tensor slot_of_row,
                        torch::Tensor cs, torch::Tensor q_out, torch::Tensor kc,
                        torch::Tensor vc, int64_t Hq, int64_t Hkv, int64_t bm, int64_t bn, int64_t var) {
  IN_BF16(x); IN_BF16(w); IN_I32(pos); IN_I32(slot_of_row); IN_BF16(cs); IN_BF16(q_out); IN_BF16(kc);
  IN_BF16(vc);
  const int K = x.size(-1), M = pos.numel(), N = (Hq + 2 * Hkv) * 256;
  TORCH_CHECK(x.numel() == (int64_t)M * K, "gemm_ring_qkv_rope: x must be [M, K] with M = pos.numel()");
  TORCH_CHECK(w.dim() == 2 && w.size(0) == N && w.size(1) == K, "gemm_ring_qkv_rope: w shape");
  TORCH_CHECK(tb_gemm_ring_ok(M, N, K, 4, (int)bm, (int)bn, (int)var), "gemm_ring_qkv_rope: unsupported tile / shape");
  TORCH_CHECK(q_out.numel() == (int64_t)M * Hq * 256, "gemm_ring_qkv_rope: q_out shape");
  TORCH_CHECK(kc.dim() == 4 && kc.size(1) == Hkv && kc.size(3) == 256 && vc.sizes() == kc.sizes(),
              "gemm_ring_qkv_rope: cache shape [slots, Hkv, S, 256]");
  TORCH_CHECK(cs.dim() == 3 && cs.size(1) == 128 && cs.size(2) == 2, "gemm_ring_qkv_rope: rope table [max_pos, 128, 2]");
  TORCH_CHECK(slot_of_row.numel() == M, "gemm_ring_qkv_rope: slot_of_row numel");
  c10::DeviceGuard g(x.device());
  tb_gemm_ring_qkv_rope(cbf(x), cbf(w), pos.data_ptr<int32_t>(), slot_of_row.data_ptr<int32_t>(), cbf(cs),
                        bf(q_out), bf(kc), bf(vc), M, K, Hq, Hkv, kc.size(2), cs.size(0),
                        (int)bm, (int)bn, (int)var, cur_stream());
}

// Split-K gemm4 (thin grids): fp32 partials of ks K ranges into ws, then the ordered reduction into C (bf16 [M, N], or
// the GeGLU [M, N/2] of the interleaved gate|up rows for epi 3).  ks <= 0: the launcher's heuristic.
// split GEMM into fp32 partials only (no reduction); returns the split count used
int64_t gemm4_splitk_part(torch::Tensor A, torch::Tensor W, torch::Tensor ws, int64_t tile_rows, int64_t ks) {
  IN_BF16(A); IN_BF16(W); IN_F32(ws);
  TORCH_CHECK(W.dim() == 2 && (tile_rows == 256 || tile_rows == 128 || tile_rows == 64),
              "gemm4_splitk_part: W [N, K], tile_rows 64|128|256");
  const int K = A.size(-1), M = A.numel() / K, N = W.size(0);
  TORCH_CHECK(W.size(1) == K && tb_gemm4_ok(M, N, K), "gemm4_splitk_part: need N % 256 == 0, K % 64 == 0");
  if (ks <= 0) ks = tb_gemm4_splitk_ks(M, N, K, tile_rows);
  const int NT = K / 64, kc = (NT + (int)ks - 1) / (int)ks, kse = (NT + kc - 1) / kc;
  TORCH_CHECK(ws.numel() >= (int64_t)kse * M * N, "gemm4_splitk_part: ws needs ks * M * N floats");
  c10::DeviceGuard g(A.device());
  return tb_gemm4_splitk_part(cbf(A), cbf(W), ws.data_ptr<float>(), M, N, K, (int)tile_rows, (int)ks, cur_stream());
}

int64_t gemm4_splitk_ks(int64_t M, int64_t N, int64_t K, int64_t tile_rows) {
  return tb_gemm4_splitk_ks(M, N, K, tile_rows);
}
void gemm4_splitk(torch::Tensor A, torch::Tensor W, torch::Tensor C, torch::Tensor ws, int64_t epi, int64_t tile_rows,
                  int64_t ks) {
  IN_BF16(A); IN_BF16(W); IN_BF16(C); IN_F32(ws);
  TORCH_CHECK(W.dim() == 2, "gemm4_splitk: W must be [N, K]");
  TORCH_CHECK(tile_rows == 256 || tile_rows == 128 || tile_rows == 64, "gemm4_splitk: tile_rows must be 64, 128 or 256");
  const int K = A.size(-1), M = A.numel() / K, N = W.size(0);
  TORCH_CHECK(W.size(1) == K, "gemm4_splitk: K mismatch");
  TORCH_CHECK(tb_gemm4_ok(M, N, K), "gemm4_splitk: need N % 256 == 0, K % 64 == 0, K >= 64");
  TORCH_CHECK(epi == 0 || epi == 3, "gemm4_splitk: epi must be 0 (bf16) or 3 (GeGLU)");
  const int64_t ncols = epi == 3 ? N / 2 : N;
  TORCH_CHECK(C.numel() == (int64_t)M * ncols, "gemm4_splitk: C shape");
  if (ks <= 0) ks = tb_gemm4_splitk_ks(M, N, K, tile_rows);
  const int NT = K / 64, kc = (NT + (int)ks - 1) / (int)ks, kse = (NT + kc - 1) / kc;
  TORCH_CHECK(ws.numel() >= (int64_t)kse * M * N, "gemm4_splitk: ws needs ks * M * N floats");
  c10::DeviceGuard g(A.device());
  tb_gemm4_splitk(cbf(A), cbf(W), reinterpret_cast<uint16_t*>(C.data_ptr()), ws.data_ptr<float>(), M, N, K, (int)ncols,
                  (int)epi, (int)tile_rows, (int)ks, cur_stream());
}

// QKV projection with RoPE + KV-cache scatter in the epilogue (gemm4.hip G4_ROPE): x [M, K] @ wqkv [(Hq+2Hkv)*256, K]^T;
// the same outputs as linear + rope_qkv_cache (head_dim 256 only), the qkv activation never reaches memory.
void gemm4_qkv_rope(torch::Tensor x, torch::Tensor w, torch::Tensor pos, torch::Tensor slot_of_row, torch::Tensor cs,
                    torch::Tensor q_out, torch::Tensor kc, torch::Tensor vc, int64_t Hq, int64_t Hkv,
                    int64_t tile_rows) {
  IN_BF16(x); IN_BF16(w); IN_I32(pos); IN_I32(slot_of_row); IN_BF16(cs); IN_BF16(q_out); IN_BF16(kc);
  IN_BF16(vc);
  const int K = x.size(-1), M = pos.numel();
  TORCH_CHECK(x.numel() == (int64_t)M * K, "gemm4_qkv_rope: x must be [M, K] with M = pos.numel()");
  TORCH_CHECK(w.dim() == 2 && w.size(0) == (Hq + 2 * Hkv) * 256 && w.size(1) == K, "gemm4_qkv_rope: w shape");
  TORCH_CHECK(tb_gemm4_ok(M, (Hq + 2 * Hkv) * 256, K), "gemm4_qkv_rope: need K % 64 == 0, K >= 64");
  TORCH_CHECK(q_out.numel() == (int64_t)M * Hq * 256, "gemm4_qkv_rope: q_out shape");
  TORCH_CHECK(kc.dim() == 4 && kc.size(1) == Hkv && kc.size(3) == 256 && vc.sizes() == kc.sizes(),
              "gemm4_qkv_rope: cache shape [slots, Hkv, S, 256]");
  TORCH_CHECK(cs.dim() == 3 && cs.size(1) == 128 && cs.size(2) == 2, "gemm4_qkv_rope: rope table [max_pos, 128, 2]");
  TORCH_CHECK(slot_of_row.numel() == M, "gemm4_qkv_rope: slot_of_row numel");
  TORCH_CHECK(tile_rows == 256 || tile_rows == 128, "gemm4_qkv_rope: tile_rows must be 256 or 128");
  c10::DeviceGuard g(x.device());
  tb_gemm4_qkv_rope(cbf(x), cbf(w), pos.data_ptr<int32_t>(), slot_of_row.data_ptr<int32_t>(), cbf(cs),
                    bf(q_out), bf(kc), bf(vc), M, K, Hq, Hkv, kc.size(2), cs.size(0),
                    (int)tile_rows, cur_stream());
}

// Row combination of fp32 rows given by device address (the sweep's lens base, elementwise.hip)
void row_combine(torch::Tensor ptr, torch::Tensor coef, torch::Tensor out) {
  CHECK_DEV(ptr); CHECK_CONTIG(ptr); IN_F32(coef); IN_F32(out);
  TORCH_CHECK(ptr.scalar_type() == at::kLong && ptr.dim() == 2 && coef.sizes() == ptr.sizes(),
              "row_combine: ptr int64 [B, T], coef f32 [B, T]");
  const int B = ptr.size(0), T = ptr.size(1), V = out.size(-1);
  TORCH_CHECK(out.numel() == (int64_t)B * V && V % 4 == 0, "row_combine: out [B, V], V % 4 == 0");
  c10::DeviceGuard g(out.device());
  tb_row_combine(ptr.data_ptr<int64_t>(), coef.data_ptr<float>(), out.data_ptr<float>(), B, T, V, cur_stream());
}

// random orthonormal bases (csrc/basis.hip) written into rows [rows[i], rows[i] + ranks[i]) of an fp32 [R, D] table
void random_basis(torch::Tensor seeds, torch::Tensor ranks, torch::Tensor rows, torch::Tensor table, int64_t qu) {
  CHECK_DEV(seeds); CHECK_CONTIG(seeds); CHECK_DEV(ranks); CHECK_CONTIG(ranks); CHECK_DEV(rows); CHECK_CONTIG(rows);
  IN_F32(table);
  TORCH_CHECK(seeds.scalar_type() == at::kLong && ranks.scalar_type() == at::kInt && rows.scalar_type() == at::kLong,
              "random_basis: seeds int64, ranks int32, rows int64");
  const int n = seeds.numel(), D = table.size(-1);
  TORCH_CHECK(ranks.numel() == n && rows.numel() == n && table.dim() == 2, "random_basis: [n] seeds/ranks/rows, [R, D] table");
  TORCH_CHECK(tb_random_basis_ok(D), "random_basis: D = ", D, " outside (0, 4096]");
  c10::DeviceGuard g(table.device());
  tb_random_basis(reinterpret_cast<const uint64_t*>(seeds.data_ptr<int64_t>()), ranks.data_ptr<int32_t>(),
                  rows.data_ptr<int64_t>(), n, D, table.data_ptr<float>(), cur_stream(), (int)qu);
}

// ---- multi-adapter LoRA (models/lora.py): two-source A operands [x (k0 columns) | T (K - k0 columns)] of the in-tree
// GEMMs (gemm4 / ring, same K chain as one [M, K] operand: batch-invariant, every fused epilogue kept) and the masked
// down-projection T = x A_all^T (only the row's adapter's columns, ring RG_LMASK)
static void l2a_check(const torch::Tensor& x, const torch::Tensor& a2, const torch::Tensor& W, int& M, int& K, int& k0) {
  IN_BF16(x); IN_BF16(a2); IN_BF16(W);
  TORCH_CHECK(W.dim() == 2, "l2a: W must be [N, K]");
  k0 = x.size(-1);
  M = x.numel() / k0;
  K = W.size(1);
  TORCH_CHECK(a2.numel() == (int64_t)M * (K - k0), "l2a: a2 must be [M, K - k0]");
  TORCH_CHECK(k0 > 0 && k0 < K && k0 % 128 == 0 && K % 128 == 0, "l2a: k0 and K must be multiples of 128, k0 < K");
}

void gemm4_l2a(torch::Tensor x, torch::Tensor a2, torch::Tensor W, torch::Tensor C, int64_t epi, int64_t tile_rows) {
  int M, K, k0;
  l2a_check(x, a2, W, M, K, k0);
  IN_BF16(C);
  const int N = W.size(0);
  TORCH_CHECK(tb_gemm4_ok(M, N, K) && (epi == 0 || epi == 3) && (tile_rows == 256 || tile_rows == 128),
              "gemm4_l2a: N % 256, epi 0 | 3, tile_rows 256 | 128");
  const int64_t ncols = epi == 3 ? N / 2 : N;
  TORCH_CHECK(C.numel() == (int64_t)M * ncols, "gemm4_l2a: C shape");
  c10::DeviceGuard g(x.device());
  tb_gemm4(cbf(x), cbf(W), C.data_ptr(), nullptr, nullptr, M, N, K, (int)ncols, (int)epi, (int)tile_rows, cur_stream(),
           cbf(a2), k0);
}

void gemm_ring_l2a(torch::Tensor x, torch::Tensor a2, torch::Tensor W, torch::Tensor C, int64_t epi, int64_t bm,
                   int64_t bn) {
  int M, K, k0;
  l2a_check(x, a2, W, M, K, k0);
  IN_BF16(C);
  const int N = W.size(0);
  TORCH_CHECK((epi == 0 || epi == 3) && tb_gemm_ring_ok(M, N, K, (int)epi, (int)bm, (int)bn, 1),
              "gemm_ring_l2a: unsupported tile / shape (144 KB ring)");
  const int64_t ncols = epi == 3 ? N / 2 : N;
  TORCH_CHECK(C.numel() == (int64_t)M * ncols, "gemm_ring_l2a: C shape");
  c10::DeviceGuard g(x.device());
  tb_gemm_ring(cbf(x), cbf(W), bf(C), M, N, K, (int)ncols, (int)epi, (int)bm, (int)bn, 1, cur_stream(), cbf(a2), k0);
}

static void qkv_l2a_check(const torch::Tensor& pos, const torch::Tensor& slot_of_row, const torch::Tensor& cs,
                          const torch::Tensor& q_out, const torch::Tensor& kc, const torch::Tensor& vc, int M, int64_t Hq,
                          int64_t Hkv, const torch::Tensor& W) {
  IN_I32(pos); IN_I32(slot_of_row); IN_BF16(cs); IN_BF16(q_out); IN_BF16(kc); IN_BF16(vc);
  TORCH_CHECK(pos.numel() == M && slot_of_row.numel() == M, "qkv_l2a: pos / slot_of_row numel");
  TORCH_CHECK(W.size(0) == (Hq + 2 * Hkv) * 256, "qkv_l2a: w rows");
  TORCH_CHECK(q_out.numel() == (int64_t)M * Hq * 256, "qkv_l2a: q_out shape");
  TORCH_CHECK(kc.dim() == 4 && kc.size(1) == Hkv && kc.size(3) == 256 && vc.sizes() == kc.sizes(),
              "qkv_l2a: cache shape [slots, Hkv, S, 256]");
  TORCH_CHECK(cs.dim() == 3 && cs.size(1) == 128 && cs.size(2) == 2, "qkv_l2a: rope table [max_pos, 128, 2]");
}

void gemm4_qkv_rope_l2a(torch::Tensor x, torch::Tensor a2, torch::Tensor w, torch::Tensor pos, torch::Tensor slot_of_row,
                        torch::Tensor cs, torch::Tensor q_out, torch::Tensor kc, torch::Tensor vc, int64_t Hq,
                        int64_t Hkv, int64_t tile_rows) {
  int M, K, k0;
  l2a_check(x, a2, w, M, K, k0);
  qkv_l2a_check(pos, slot_of_row, cs, q_out, kc, vc, M, Hq, Hkv, w);
  TORCH_CHECK(tile_rows == 256 || tile_rows == 128, "gemm4_qkv_rope_l2a: tile_rows must be 256 or 128");
  c10::DeviceGuard g(x.device());
  tb_gemm4_qkv_rope(cbf(x), cbf(w), pos.data_ptr<int32_t>(), slot_of_row.data_ptr<int32_t>(), cbf(cs), bf(q_out),
                    bf(kc), bf(vc), M, K, Hq, Hkv, kc.size(2), cs.size(0), (int)tile_rows, cur_stream(), cbf(a2), k0);
}

void gemm_ring_qkv_rope_l2a(torch::Tensor x, torch::Tensor a2, torch::Tensor w, torch::Tensor pos,
                            torch::Tensor slot_of_row, torch::Tensor cs, torch::Tensor q_out, torch::Tensor kc,
                            torch::Tensor vc, int64_t Hq, int64_t Hkv, int64_t bm, int64_t bn) {
  int M, K, k0;
  l2a_check(x, a2, w, M, K, k0);
  qkv_l2a_check(pos, slot_of_row, cs, q_out, kc, vc, M, Hq, Hkv, w);
  TORCH_CHECK(tb_gemm_ring_ok(M, w.size(0), K, 4, (int)bm, (int)bn, 1), "gemm_ring_qkv_rope_l2a: unsupported tile");
  c10::DeviceGuard g(x.device());
  tb_gemm_ring_qkv_rope(cbf(x), cbf(w), pos.data_ptr<int32_t>(), slot_of_row.data_ptr<int32_t>(), cbf(cs), bf(q_out),
                        bf(kc), bf(vc), M, K, Hq, Hkv, kc.size(2), cs.size(0), (int)bm, (int)bn, 1, cur_stream(),
                        cbf(a2), k0);
}

// T [M, N] = the row's adapter's columns of x A_all^T (A_all [N, K] = the bank's stacked down-projections, zero-padded
// rows), every other column 0; adapter [M] int32 (-1: base model, T = 0).  T may be wider (row stride ldt >= N): its
// columns >= N are not written.
// part: empty (one workgroup per tile, chunks folded in registers) or fp32 [tb_lora_t_chunks(K), M, N] (one workgroup
// per (tile, chunk) + the ordered fold kernel); both forms give the same bits
void lora_t(torch::Tensor x, torch::Tensor a_all, torch::Tensor t, torch::Tensor adapter, int64_t nsr, int64_t nr,
            int64_t r, int64_t bm, int64_t bn, torch::Tensor part) {
  IN_BF16(x); IN_BF16(a_all); IN_BF16(t); IN_I32(adapter);
  const int K = x.size(-1), M = x.numel() / K, N = a_all.size(0);
  TORCH_CHECK(a_all.dim() == 2 && a_all.size(1) == K, "lora_t: A_all must be [N, K]");
  const int ldt = t.size(-1);
  TORCH_CHECK(ldt >= N && t.numel() == (int64_t)M * ldt && adapter.numel() == M, "lora_t: T [M, >= N], adapter [M]");
  TORCH_CHECK(nsr <= N && nr > 0 && r > 0 && nr % r == 0, "lora_t: widths");
  TORCH_CHECK(tb_lora_t_ok(M, N, K, (int)bm, (int)bn), "lora_t: unsupported tile / shape");
  float* pp = nullptr;
  if (part.numel() > 0) {
    IN_F32(part);
    TORCH_CHECK(part.numel() == (int64_t)tb_lora_t_chunks(K) * M * N, "lora_t: part must be [chunks(K), M, N]");
    pp = part.data_ptr<float>();
  }
  c10::DeviceGuard g(x.device());
  tb_lora_t(cbf(x), cbf(a_all), bf(t), adapter.data_ptr<int32_t>(), M, N, K, (int)nsr, (int)nr, (int)r, (int)bm,
            (int)bn, cur_stream(), ldt, pp);
}

int64_t lora_t_chunks(int64_t K) { return tb_lora_t_chunks((int)K); }

bool lora_t_ok(int64_t M, int64_t N, int64_t K, int64_t bm, int64_t bn) {
  return tb_lora_t_ok((int)M, (int)N, (int)K, (int)bm, (int)bn);
}

// Logit-lens unembedding on the four-wave GEMM (gemm4.hip G4_LENS): bf16 logits and their per-row
// log-sum-exp (no softcap), so the lens needs no separate row_lse pass.  part: f32 >= M * (V / 128) * 4.
void lens_gemm(torch::Tensor x, torch::Tensor W, torch::Tensor logits, torch::Tensor part, torch::Tensor lse) {
  IN_BF16(x); IN_BF16(W); IN_BF16(logits); IN_F32(part); IN_F32(lse);
  TORCH_CHECK(W.dim() == 2, "lens_gemm: W must be [V, K]");
  const int K = x.size(-1), M = x.numel() / K, N = W.size(0);
  TORCH_CHECK(W.size(1) == K, "lens_gemm: K mismatch");
  TORCH_CHECK(tb_gemm4_ok(M, N, K), "lens_gemm: need V % 256 == 0, K % 64 == 0, K >= 64");
  TORCH_CHECK(logits.numel() == (int64_t)M * N, "lens_gemm: logits shape");
  TORCH_CHECK(part.numel() >= (int64_t)M * (N / 128) * 4 && lse.numel() == M, "lens_gemm: part / lse shapes");
  c10::DeviceGuard g(x.device());
  tb_lens_gemm4(cbf(x), cbf(W), bf(logits), part.data_ptr<float>(), lse.data_ptr<float>(), M, N, K, cur_stream());
}

// Fused vocab head (gemm4.hip G4_HEAD, compact exact softcap, + head_merge): x [M, K] final-normed rows,
// W = lm_head [V, K]; the decode_head outputs (greedy token, its NLL, optional teacher-target NLL) with no
// logits in HBM.
// part: f32 workspace >= M * (V / 128) * 4; tgt_logit: f32 [M] (with tgt).
void head_fused(torch::Tensor x, torch::Tensor W, torch::Tensor part, double cap, c10::optional<torch::Tensor> tgt,
                c10::optional<torch::Tensor> tgt_logit, torch::Tensor nxt, torch::Tensor nll_self,
                c10::optional<torch::Tensor> nll_tgt) {
  IN_BF16(x); IN_BF16(W); IN_F32(part); IN_I32(nxt); IN_F32(nll_self);
  TORCH_CHECK(W.dim() == 2, "head_fused: W must be [V, K]");
  const int K = x.size(-1), M = x.numel() / K, N = W.size(0);
  TORCH_CHECK(W.size(1) == K, "head_fused: K mismatch");
  TORCH_CHECK(tb_gemm4_ok(M, N, K), "head_fused: need V % 256 == 0, K % 64 == 0, K >= 64");
  TORCH_CHECK(part.numel() >= (int64_t)M * (N / 128) * 4, "head_fused: part workspace too small");
  TORCH_CHECK(nxt.numel() == M && nll_self.numel() == M, "head_fused: output shapes");
  TORCH_CHECK(tgt.has_value() == nll_tgt.has_value() && tgt.has_value() == tgt_logit.has_value(),
              "head_fused: tgt, tgt_logit and nll_tgt go together");
  const int32_t* tp = nullptr;
  float *tl = nullptr, *np = nullptr;
  if (tgt.has_value()) {
    IN_I32((*tgt)); IN_F32((*tgt_logit)); IN_F32((*nll_tgt));
    TORCH_CHECK(tgt->numel() == M && tgt_logit->numel() == M && nll_tgt->numel() == M, "head_fused teacher shapes");
    tp = tgt->data_ptr<int32_t>();
    tl = tgt_logit->data_ptr<float>();
    np = nll_tgt->data_ptr<float>();
  }
  c10::DeviceGuard g(x.device());
  if (cap > 0) {
    const uint16_t* ct = nullptr;
    int lo = 0, hi = 0;
    float sat = 0.f;
    TORCH_CHECK(tb_softcap_compact_params((float)cap, &ct, &lo, &hi, &sat) && hi - lo <= 2048,
                "head_fused: no compact softcap registered for this cap on this device");
  }
  tb_head_fused4(cbf(x), cbf(W), part.data_ptr<float>(), (float)cap, tp, tl, nxt.data_ptr<int32_t>(),
                 nll_self.data_ptr<float>(), np, M, N, K, cur_stream());
}

void lowrank_edit(torch::Tensor h, c10::optional<torch::Tensor> x_next, torch::Tensor apply, torch::Tensor idx,
                  torch::Tensor cnt, torch::Tensor E, torch::Tensor Dm, c10::optional<torch::Tensor> bias,
                  c10::optional<torch::Tensor> thr, c10::optional<torch::Tensor> pre_bias, double alpha,
                  c10::optional<torch::Tensor> w_next, double eps, c10::optional<torch::Tensor> coef_out) {
  IN_BF16(h); IN_U8(apply); IN_I32(idx); IN_I32(cnt); CHECK_DEV(E); CHECK_CONTIG(E); CHECK_DEV(Dm);
  CHECK_CONTIG(Dm);
  TORCH_CHECK(E.scalar_type() == Dm.scalar_type(), "E/D dtype mismatch");
  const bool f32 = E.scalar_type() == at::kFloat;
  TORCH_CHECK(f32 || E.scalar_type() == at::kBFloat16, "table dtype");
  const int D = h.size(-1), M = h.numel() / D;
  TORCH_CHECK(E.size(1) == D && Dm.size(1) == D && apply.numel() == M && cnt.numel() == M, "lowrank shapes");
  TORCH_CHECK(D % 8 == 0 && D <= 256 * 8 * 4, "lowrank_edit: need D % 8 == 0 and D <= 8192");
  const int mmax = idx.numel() / M;
  TORCH_CHECK(mmax >= 1 && mmax <= 256, "lowrank mmax");
  TORCH_CHECK(!bias.has_value() || !bias->defined() || bias->numel() == E.size(0), "lowrank_edit: bias numel");
  TORCH_CHECK(!thr.has_value() || !thr->defined() || thr->numel() == E.size(0), "lowrank_edit: thr numel");
  TORCH_CHECK(!pre_bias.has_value() || !pre_bias->defined() || pre_bias->numel() == D, "lowrank_edit: pre_bias");
  if (debug_checks() && idx.numel() > 0) {   // device sync: debug builds / tests only
    // only the entries the kernel reads: rows with apply set, their first cnt ids
    const auto used = apply.to(at::kBool).view({M, 1}) &
                      (at::arange(mmax, idx.options().dtype(at::kInt)).view({1, mmax}) < cnt.view({M, 1}));
    const auto ids = idx.view({M, mmax}).masked_select(used);
    if (ids.numel() > 0)
      TORCH_CHECK(ids.min().item<int32_t>() >= 0 && ids.max().item<int32_t>() < std::min(E.size(0), Dm.size(0)),
                  "lowrank_edit: idx out of range of the E/D tables");
  }
  uint16_t* xn = nullptr;
  const uint16_t* wn = nullptr;
  if (x_next.has_value() && x_next->defined()) {
    IN_BF16((*x_next));
    TORCH_CHECK(w_next.has_value() && w_next->defined(), "x_next needs w_next");
    xn = reinterpret_cast<uint16_t*>(x_next->data_ptr());
    wn = reinterpret_cast<const uint16_t*>(w_next->data_ptr());
  }
  float* co = nullptr;
  if (coef_out.has_value() && coef_out->defined()) {
    IN_F32((*coef_out));
    co = coef_out->data_ptr<float>();
  }
  c10::DeviceGuard g(h.device());
  tb_lowrank_edit(bf(h), xn, reinterpret_cast<const uint8_t*>(apply.data_ptr()), idx.data_ptr<int32_t>(),
                  cnt.data_ptr<int32_t>(), mmax, E.data_ptr(), Dm.data_ptr(), f32 ? 1 : 0, optf(bias), optf(thr),
                  optf(pre_bias), (float)alpha, wn, (float)eps, M, D, co, cur_stream());
}

void sae_decode_sparse(torch::Tensor acts, torch::Tensor Wdec, c10::optional<torch::Tensor> b_dec,
                       c10::optional<torch::Tensor> out_bf16, c10::optional<torch::Tensor> out_f32) {
  IN_F32(acts); CHECK_DEV(Wdec); CHECK_CONTIG(Wdec);
  const bool f32 = Wdec.scalar_type() == at::kFloat;
  TORCH_CHECK(f32 || Wdec.scalar_type() == at::kBFloat16, "sae_decode_sparse: W_dec must be fp32 or bf16");
  const int L = Wdec.size(0), D = Wdec.size(1), M = acts.numel() / L;
  TORCH_CHECK(D % 8 == 0, "sae_decode_sparse: D must be a multiple of 8");
  TORCH_CHECK(acts.size(-1) == L, "sae_decode_sparse: acts last dim must equal W_dec rows");
  TORCH_CHECK(!b_dec.has_value() || !b_dec->defined() || b_dec->numel() == D, "sae_decode_sparse: b_dec numel");
  uint16_t* ob = nullptr;
  float* of = nullptr;
  if (out_bf16.has_value() && out_bf16->defined()) {
    TORCH_CHECK(out_bf16->numel() == (int64_t)M * D, "sae_decode_sparse: out_bf16 shape");
  }
  if (out_f32.has_value() && out_f32->defined()) {
    TORCH_CHECK(out_f32->numel() == (int64_t)M * D, "sae_decode_sparse: out_f32 shape");
  }
  if (out_bf16.has_value() && out_bf16->defined()) { IN_BF16((*out_bf16)); ob = reinterpret_cast<uint16_t*>(out_bf16->data_ptr()); }
  if (out_f32.has_value() && out_f32->defined()) { IN_F32((*out_f32)); of = out_f32->data_ptr<float>(); }
  c10::DeviceGuard g(acts.device());
  tb_sae_decode_sparse(acts.data_ptr<float>(), Wdec.data_ptr(), f32 ? 1 : 0, optf(b_dec), ob, of, M, L, D,
                       cur_stream());
}

void latent_score(torch::Tensor acts, torch::Tensor p, torch::Tensor spike, torch::Tensor seg, torch::Tensor out,
                  c10::optional<torch::Tensor> spike_mean, c10::optional<torch::Tensor> corr) {
  IN_F32(acts); IN_F32(p); IN_U8(spike); IN_I32(seg); IN_F32(out);
  const int L = acts.size(-1), G = seg.numel() - 1;
  TORCH_CHECK(out.numel() == (int64_t)G * L, "latent_score out");
  float* sm = nullptr;
  float* co = nullptr;
  if (spike_mean.has_value() && spike_mean->defined()) sm = spike_mean->data_ptr<float>();
  if (corr.has_value() && corr->defined()) co = corr->data_ptr<float>();
  c10::DeviceGuard g(acts.device());
  tb_latent_score(acts.data_ptr<float>(), p.data_ptr<float>(), reinterpret_cast<const uint8_t*>(spike.data_ptr()),
                  seg.data_ptr<int32_t>(), out.data_ptr<float>(), sm, co, G, L, cur_stream());
}

int64_t attention_lds_bytes(int64_t hd) { return tb_attention_lds_bytes((int)hd); }

// ---- one-shot P2P all-reduce (p2p.hip): regions are raw device pointers passed as int64
int64_t p2p_alloc(int64_t bytes, bool uncached) {
  void* p = tb_p2p_alloc((size_t)bytes, uncached ? 1 : 0);
  TORCH_CHECK(p != nullptr, "p2p_alloc: device allocation of ", bytes, " bytes failed");
  return reinterpret_cast<int64_t>(p);
}

void p2p_free(int64_t p) { TORCH_CHECK(tb_p2p_free(reinterpret_cast<void*>(p)) == 0, "p2p_free failed"); }

py::bytes p2p_get_handle(int64_t p) {
  std::string h((size_t)tb_p2p_handle_size(), '\0');
  const int e = tb_p2p_get_handle(reinterpret_cast<void*>(p), &h[0]);
  TORCH_CHECK(e == 0, "hipIpcGetMemHandle failed (hipError ", e, ")");
  return py::bytes(h);
}

int64_t p2p_open_handle(py::bytes handle) {
  std::string h = handle;
  TORCH_CHECK((int)h.size() == tb_p2p_handle_size(), "p2p_open_handle: bad handle size");
  void* p = tb_p2p_open_handle(h.data());
  TORCH_CHECK(p != nullptr, "hipIpcOpenMemHandle failed");
  return reinterpret_cast<int64_t>(p);
}

void p2p_close_handle(int64_t p) { TORCH_CHECK(tb_p2p_close_handle(reinterpret_cast<void*>(p)) == 0, "p2p_close failed"); }

void p2p_allreduce(std::vector<int64_t> bases, int64_t rank, torch::Tensor in, torch::Tensor out, int64_t blocks,
                   int64_t spin_max, bool barriers) {
  CHECK_DEV(in); CHECK_CONTIG(in); CHECK_DEV(out); CHECK_CONTIG(out);
  const bool is_bf16 = in.scalar_type() == at::kBFloat16;
  TORCH_CHECK(is_bf16 || in.scalar_type() == at::kFloat, "p2p_allreduce: bf16 or fp32");
  TORCH_CHECK(out.scalar_type() == in.scalar_type() && out.numel() == in.numel(), "p2p_allreduce: out mismatch");
  const int world = (int)bases.size();
  TORCH_CHECK(world >= 1 && world <= tb_p2p_max_ranks() && rank >= 0 && rank < world, "p2p_allreduce: ranks");
  std::vector<void*> b(world);
  for (int r = 0; r < world; ++r) b[r] = reinterpret_cast<void*>(bases[r]);
  c10::DeviceGuard g(in.device());
  const size_t nbytes = (size_t)in.numel() * in.element_size();
  const int e = tb_p2p_allreduce(b.data(), (int)rank, world, in.data_ptr(), out.data_ptr(), nbytes, is_bf16 ? 1 : 0,
                                 (int)blocks, (int)spin_max, barriers ? 1 : 0, cur_stream());
  TORCH_CHECK(e == 0, "p2p_allreduce launch failed (", e, ")");
}

void p2p_allgather(std::vector<int64_t> bases, int64_t rank, torch::Tensor in, torch::Tensor out, int64_t blocks,
                   int64_t spin_max, bool barriers) {
  CHECK_DEV(in); CHECK_CONTIG(in); CHECK_DEV(out); CHECK_CONTIG(out);
  const int world = (int)bases.size();
  TORCH_CHECK(world >= 1 && world <= tb_p2p_max_ranks() && rank >= 0 && rank < world, "p2p_allgather: ranks");
  const size_t nbytes = (size_t)in.numel() * in.element_size();
  TORCH_CHECK(nbytes % 16 == 0, "p2p_allgather: bytes must be a multiple of 16");
  TORCH_CHECK(out.scalar_type() == in.scalar_type() && out.numel() == in.numel() * world, "p2p_allgather: out must be [world, *in]");
  std::vector<void*> b(world);
  for (int r = 0; r < world; ++r) b[r] = reinterpret_cast<void*>(bases[r]);
  c10::DeviceGuard g(in.device());
  const int e = tb_p2p_allgather(b.data(), (int)rank, world, in.data_ptr(), out.data_ptr(), nbytes, (int)blocks,
                                 (int)spin_max, barriers ? 1 : 0, cur_stream());
  TORCH_CHECK(e == 0, "p2p_allgather launch failed (", e, ")");
}

void slot_copy(torch::Tensor dst, torch::Tensor src, torch::Tensor dslot, torch::Tensor sslot, int64_t dst_l0,
               int64_t src_l0, int64_t nl) {
  IN_BF16(dst); IN_BF16(src); IN_I32(dslot); IN_I32(sslot);
  TORCH_CHECK(dst.dim() >= 3 && src.dim() == dst.dim(), "slot_copy: [L, slots, ...] tensors");
  const int64_t inner = dst.numel() / (dst.size(0) * dst.size(1));
  TORCH_CHECK(src.numel() / (src.size(0) * src.size(1)) == inner && inner % 8 == 0, "slot_copy: slot size");
  TORCH_CHECK(dslot.numel() == sslot.numel(), "slot_copy: index lists");
  TORCH_CHECK(nl >= 0 && dst_l0 >= 0 && src_l0 >= 0 && dst_l0 + nl <= dst.size(0) && src_l0 + nl <= src.size(0),
              "slot_copy: layer range");
  const int n = dslot.numel();
  if (n == 0 || nl == 0) return;
  // (slot ranges are checked on the host lists by ops.slot_copy: no device sync here)
  c10::DeviceGuard g(dst.device());
  tb_slot_copy(bf(dst), bf(src), dslot.data_ptr<int32_t>(), sslot.data_ptr<int32_t>(), n, (int)nl, inner,
               dst.size(1), src.size(1), (int)dst_l0, (int)src_l0, cur_stream());
}

// vocab-parallel merges (csrc/vp.hip)
void vp_head_merge(torch::Tensor st, c10::optional<torch::Tensor> tgt, int64_t V, c10::optional<torch::Tensor> nxt,
                   c10::optional<torch::Tensor> nll_self, c10::optional<torch::Tensor> nll_tgt) {
  IN_F32(st);
  TORCH_CHECK(st.dim() == 3 && st.size(2) == 4, "vp_head_merge: st must be [tp, R, 4]");
  const int tp = st.size(0), R = st.size(1);
  auto chk = [&](const c10::optional<torch::Tensor>& t, bool i32) {
    if (!t) return;
    if (i32) { IN_I32((*t)); } else { IN_F32((*t)); }
    TORCH_CHECK(t->numel() == R, "vp_head_merge: per-row output size");
  };
  chk(tgt, true); chk(nxt, true); chk(nll_self, false); chk(nll_tgt, false);
  c10::DeviceGuard g(st.device());
  tb_vp_head_merge(st.data_ptr<float>(), tp, R, tgt ? tgt->data_ptr<int32_t>() : nullptr, (int)V,
                   nxt ? nxt->data_ptr<int32_t>() : nullptr, nll_self ? nll_self->data_ptr<float>() : nullptr,
                   nll_tgt ? nll_tgt->data_ptr<float>() : nullptr, cur_stream());
}

void vp_lse_merge(torch::Tensor lse, torch::Tensor out) {
  IN_F32(lse); IN_F32(out);
  TORCH_CHECK(lse.dim() == 2 && out.numel() == lse.size(1), "vp_lse_merge: lse [tp, R] -> out [R]");
  c10::DeviceGuard g(lse.device());
  tb_vp_lse_merge(lse.data_ptr<float>(), lse.size(0), lse.size(1), out.data_ptr<float>(), cur_stream());
}

void vp_topk_merge(torch::Tensor vals, torch::Tensor ids, torch::Tensor ov, torch::Tensor oi) {
  IN_F32(vals); IN_I32(ids); IN_F32(ov); IN_I32(oi);
  TORCH_CHECK(vals.dim() == 3 && ids.sizes() == vals.sizes(), "vp_topk_merge: vals/ids [tp, n, k]");
  const int tp = vals.size(0), n = vals.size(1), k = vals.size(2);
  TORCH_CHECK(k >= 1 && k <= 64 && ov.numel() == (int64_t)n * k && oi.numel() == (int64_t)n * k, "vp_topk_merge: k");
  c10::DeviceGuard g(vals.device());
  tb_vp_topk_merge(vals.data_ptr<float>(), ids.data_ptr<int32_t>(), tp, n, k, ov.data_ptr<float>(),
                   oi.data_ptr<int32_t>(), cur_stream());
}

int64_t p2p_read_error(int64_t own) { return (int64_t)tb_p2p_read_error(reinterpret_cast<void*>(own)); }
#define IN_I64(t) CHECK_DEV(t); CHECK_CONTIG(t); TORCH_CHECK((t).scalar_type() == at::kLong, #t " must be int64")

// decode-step bookkeeping (csrc/decode_step.hip): the first nb rows of the generator's [B, ...] state buffers
void decode_pre(torch::Tensor step_idx, torch::Tensor tf_tgt, torch::Tensor tf_step, int64_t nb) {
  IN_I64(step_idx); IN_I32(tf_tgt); IN_I32(tf_step);
  TORCH_CHECK(tf_tgt.dim() == 2 && nb >= 0 && nb <= tf_tgt.size(0) && step_idx.numel() >= nb && tf_step.numel() >= nb,
              "decode_pre shapes");
  c10::DeviceGuard g(tf_tgt.device());
  tb_decode_pre(step_idx.data_ptr<int64_t>(), tf_tgt.data_ptr<int32_t>(), tf_step.data_ptr<int32_t>(), (int)nb,
                (int)tf_tgt.size(1), cur_stream());
}

void decode_post(torch::Tensor nxt, torch::Tensor nll, torch::Tensor tf_nll, torch::Tensor done, torch::Tensor step_idx,
                 torch::Tensor out_tok, torch::Tensor out_nll, torch::Tensor out_tf_nll, torch::Tensor stop,
                 torch::Tensor tok, torch::Tensor pos, int64_t nb, int64_t pad) {
  IN_I32(nxt); IN_F32(nll); IN_F32(tf_nll); IN_U8(done); IN_I64(step_idx); IN_I32(out_tok); IN_F32(out_nll);
  IN_F32(out_tf_nll); IN_I32(stop); IN_I32(tok); IN_I32(pos);
  const int64_t W = out_tok.size(1);
  TORCH_CHECK(out_tok.dim() == 2 && out_nll.sizes() == out_tok.sizes() && out_tf_nll.sizes() == out_tok.sizes() &&
              nb >= 0 && nb <= out_tok.size(0), "decode_post: output shapes");
  for (const auto* t : {&nxt, &nll, &tf_nll, &done, &step_idx, &tok, &pos})
    TORCH_CHECK(t->numel() >= nb, "decode_post: per-row buffer shorter than nb");
  c10::DeviceGuard g(nxt.device());
  tb_decode_post(nxt.data_ptr<int32_t>(), nll.data_ptr<float>(), tf_nll.data_ptr<float>(),
                 reinterpret_cast<uint8_t*>(done.data_ptr()), step_idx.data_ptr<int64_t>(), out_tok.data_ptr<int32_t>(),
                 out_nll.data_ptr<float>(), out_tf_nll.data_ptr<float>(), stop.data_ptr<int32_t>(), (int)stop.numel(),
                 tok.data_ptr<int32_t>(), pos.data_ptr<int32_t>(), (int)nb, (int)W, (int)pad, cur_stream());
}

void share_lo_gather(torch::Tensor rep, torch::Tensor U, torch::Tensor tok, torch::Tensor pos, torch::Tensor slot,
                     torch::Tensor s_tok, torch::Tensor s_pos, torch::Tensor s_slot, c10::optional<torch::Tensor> kp_slot,
                     c10::optional<torch::Tensor> kp_len_lo, c10::optional<torch::Tensor> l_slot,
                     c10::optional<torch::Tensor> l_len_lo, int64_t nb, int64_t S) {
  IN_I64(rep); IN_I64(U); IN_I32(tok); IN_I32(pos); IN_I32(slot); IN_I32(s_tok); IN_I32(s_pos); IN_I32(s_slot);
  const int64_t B = tok.numel();
  TORCH_CHECK(nb >= 0 && nb <= B && rep.numel() >= nb && pos.numel() == B && slot.numel() == B &&
              s_tok.numel() >= nb && s_pos.numel() >= nb && s_slot.numel() >= nb && U.numel() == 1,
              "share_lo_gather shapes");
  const bool kp = kp_slot.has_value() && kp_slot->defined();
  const int32_t *ks = nullptr, *kl = nullptr;
  int32_t *ls = nullptr, *ll = nullptr;
  if (kp) {
    TORCH_CHECK(kp_len_lo.has_value() && l_slot.has_value() && l_len_lo.has_value(), "share_lo_gather: prefix set");
    IN_I32((*kp_slot)); IN_I32((*kp_len_lo)); IN_I32((*l_slot)); IN_I32((*l_len_lo));
    TORCH_CHECK(kp_slot->numel() == B && kp_len_lo->numel() == B && l_slot->numel() >= nb && l_len_lo->numel() >= nb,
                "share_lo_gather: prefix shapes");
    ks = kp_slot->data_ptr<int32_t>(); kl = kp_len_lo->data_ptr<int32_t>();
    ls = l_slot->data_ptr<int32_t>(); ll = l_len_lo->data_ptr<int32_t>();
  }
  c10::DeviceGuard g(tok.device());
  tb_share_lo_gather(rep.data_ptr<int64_t>(), U.data_ptr<int64_t>(), tok.data_ptr<int32_t>(), pos.data_ptr<int32_t>(),
                     slot.data_ptr<int32_t>(), s_tok.data_ptr<int32_t>(), s_pos.data_ptr<int32_t>(),
                     s_slot.data_ptr<int32_t>(), ks, kl, ls, ll, (int)nb, (int)B, (int)S, cur_stream());
}

void capture_rows(torch::Tensor store, torch::Tensor h, torch::Tensor pos, torch::Tensor slot, int64_t T) {
  IN_BF16(store); IN_BF16(h); IN_I32(pos); IN_I32(slot);
  TORCH_CHECK(store.dim() == 3 && h.size(-1) == store.size(2) && store.size(2) % 8 == 0, "capture_rows: shapes");
  const int64_t D = store.size(2), n = h.numel() / D;
  TORCH_CHECK(T >= 1 && n % T == 0 && pos.numel() == n && slot.numel() >= n / T, "capture_rows: rows / pos / slot");
  if (debug_checks() && n > 0) {
    const auto sl = slot.narrow(0, 0, n / T);
    TORCH_CHECK(sl.min().item<int>() >= 0 && sl.max().item<int>() < store.size(0), "capture_rows: slot out of range");
  }
  c10::DeviceGuard g(h.device());
  tb_capture_rows(bf(store), cbf(h), pos.data_ptr<int32_t>(), slot.data_ptr<int32_t>(), (int)n, (int)T,
                  (int)store.size(1), (int)D, cur_stream());
}

void row_gather(torch::Tensor src, torch::Tensor idx, torch::Tensor out) {
  IN_BF16(src); IN_BF16(out); CHECK_DEV(idx); CHECK_CONTIG(idx);
  TORCH_CHECK(idx.scalar_type() == at::kLong || idx.scalar_type() == at::kInt, "row_gather: idx int32/int64");
  const int64_t D = src.size(-1), n = idx.numel();
  TORCH_CHECK(D % 8 == 0 && out.size(-1) == D && out.numel() >= n * D, "row_gather: shapes");
  if (debug_checks() && n > 0)
    TORCH_CHECK(idx.min().item<int64_t>() >= 0 && idx.max().item<int64_t>() < src.numel() / D,
                "row_gather: index out of range");
  c10::DeviceGuard g(src.device());
  tb_row_gather(bf(out), cbf(src), idx.data_ptr(), idx.scalar_type() == at::kLong, (int)n, (int)D, cur_stream());
}

void share_group(torch::Tensor gid, torch::Tensor tok, torch::Tensor rep, torch::Tensor grp, torch::Tensor src,
                 torch::Tensor U, int64_t nb, int64_t act, bool first, int64_t V) {
  IN_I64(gid); IN_I32(tok); IN_I64(rep); IN_I64(grp); IN_I32(src); IN_I64(U);
  TORCH_CHECK(nb >= 0 && nb <= tb_share_group_max_rows() && gid.numel() >= nb && tok.numel() >= nb &&
              rep.numel() >= nb && grp.numel() >= nb && src.numel() >= nb && U.numel() == 1, "share_group shapes");
  c10::DeviceGuard g(gid.device());
  tb_share_group(gid.data_ptr<int64_t>(), tok.data_ptr<int32_t>(), rep.data_ptr<int64_t>(), grp.data_ptr<int64_t>(),
                 src.data_ptr<int32_t>(), U.data_ptr<int64_t>(), (int)nb, (int)act, first ? 1 : 0, V, cur_stream());
}
int64_t share_group_max_rows() { return tb_share_group_max_rows(); }

int64_t p2p_header_bytes() { return tb_p2p_header_bytes(); }
int64_t p2p_max_ranks() { return tb_p2p_max_ranks(); }

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "taboo_brittleness_amd gfx950 kernels";
  m.def("rmsnorm", &rmsnorm);
  m.def("add_rmsnorm2", &add_rmsnorm2);
  m.def("embed_rmsnorm", &embed_rmsnorm);
  m.def("rope_qkv_cache", &rope_qkv_cache);
  m.def("rope_qkv_cache_part", &rope_qkv_cache_part);
  m.def("kv_fanout", &kv_fanout);
  m.def("decode_pre", &decode_pre);
  m.def("decode_post", &decode_post);
  m.def("share_lo_gather", &share_lo_gather);
  m.def("capture_rows", &capture_rows);
  m.def("row_gather", &row_gather);
  m.def("share_group", &share_group);
  m.def("share_group_max_rows", &share_group_max_rows);
  m.def("attention_split_rows", [](int64_t n, bool prefix) { return (int64_t)tb_attention_split_rows((int)n, prefix); });
  m.def("attention", &attention);
  m.def("attention_prefix", &attention_prefix);
  m.def("attention_varlen", &attention_varlen);
  m.def("attention_varlen_prefix", &attention_varlen_prefix);
  m.def("geglu", &geglu);
  m.def("argmax_rows", &argmax_rows);
  m.def("row_lse", &row_lse);
  m.def("gather_probs", &gather_probs);
  m.def("lens_colsum", &lens_colsum);
  m.def("topk_rows", &topk_rows);
  m.def("xent_rows", &xent_rows);
  m.def("decode_head", &decode_head);
  m.def("decode_head_stats", &decode_head_stats);
  m.def("register_softcap_table", &register_softcap_table);
  m.def("register_softcap_compact", &register_softcap_compact);
  m.def("softcap_compact", &softcap_compact);
  m.def("gemm_nt", &gemm_nt);
  m.def("gemm4", &gemm4);
  m.def("gemm4_ok", &gemm4_ok);
  m.def("gemm_ring", &gemm_ring);
  m.def("gemm_ring_ok", &gemm_ring_ok);
  m.def("gemm_ring_tiles", &gemm_ring_tiles);
  m.def("gemm_ring_qkv_rope", &gemm_ring_qkv_rope);
  m.def("gemm4_splitk", &gemm4_splitk);
  m.def("gemm4_splitk_ks", &gemm4_splitk_ks);
  m.def("gemm4_splitk_part", &gemm4_splitk_part);
  m.def("add_rmsnorm2_part", &add_rmsnorm2_part);
  m.def("gemm4_qkv_rope", &gemm4_qkv_rope);
  m.def("gemm4_l2a", &gemm4_l2a);
  m.def("gemm_ring_l2a", &gemm_ring_l2a);
  m.def("gemm4_qkv_rope_l2a", &gemm4_qkv_rope_l2a);
  m.def("gemm_ring_qkv_rope_l2a", &gemm_ring_qkv_rope_l2a);
  m.def("lora_t", &lora_t);
  m.def("lora_t_chunks", &lora_t_chunks);
  m.def("row_combine", &row_combine);
  m.def("random_basis", &random_basis);
  m.def("lora_t_ok", &lora_t_ok);
  m.def("head_fused", &head_fused);
  m.def("lens_gemm", &lens_gemm);
  m.def("lowrank_edit", &lowrank_edit);
  m.def("sae_decode_sparse", &sae_decode_sparse);
  m.def("latent_score", &latent_score);
  m.def("attention_lds_bytes", &attention_lds_bytes);
  m.def("p2p_alloc", &p2p_alloc);
  m.def("p2p_free", &p2p_free);
  m.def("p2p_get_handle", &p2p_get_handle);
  m.def("p2p_open_handle", &p2p_open_handle);
  m.def("p2p_close_handle", &p2p_close_handle);
  m.def("p2p_allreduce", &p2p_allreduce);
  m.def("p2p_allgather", &p2p_allgather);
  m.def("vp_head_merge", &vp_head_merge);
  m.def("slot_copy", &slot_copy);
  m.def("vp_lse_merge", &vp_lse_merge);
  m.def("vp_topk_merge", &vp_topk_merge);
  m.def("p2p_read_error", &p2p_read_error);
  m.def("p2p_header_bytes", &p2p_header_bytes);
  m.def("p2p_max_ranks", &p2p_max_ranks);
}
