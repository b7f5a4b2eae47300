// Host launchers for the gfx950 kernels.  Raw pointers + stream only, so the
// .hip translation units never include the (slow to compile) torch headers;
// bindings.cpp does the tensor checks and passes the current HIP stream.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// norm.hip
void tb_rmsnorm(const uint16_t* x, const uint16_t* w, uint16_t* y, int M, int D, float eps, hipStream_t st);
void tb_add_rmsnorm2(uint16_t* h, const uint16_t* o, const uint16_t* w_post, const uint16_t* w_next, uint16_t* x,
                     int M, int D, float eps, hipStream_t st);
void tb_embed_rmsnorm(const int32_t* ids, const uint16_t* E, const uint16_t* w, uint16_t* h, uint16_t* x, int M,
                      int D, int V, float scale, float eps, hipStream_t st);
// rope.hip
void tb_rope_qkv_cache(const uint16_t* qkv, const int32_t* pos, const int32_t* slot_of_row, const float* cos_t,
                       const float* sin_t, uint16_t* q_out, uint16_t* kc, uint16_t* vc, int M, int Hq, int Hkv,
                       int HD, int S, int max_pos, hipStream_t st);
// the same from the ks fp32 split-K partials [ks, M, (Hq + 2 Hkv) HD] of the QKV projection (summed in order, bf16)
void tb_rope_qkv_cache_part(const float* part, int ks, const int32_t* pos, const int32_t* slot_of_row,
                            const float* cos_t, const float* sin_t, uint16_t* q_out, uint16_t* kc, uint16_t* vc, int M,
                            int Hq, int Hkv, int HD, int S, int max_pos, hipStream_t st);
void tb_kv_fanout(uint16_t* kc, uint16_t* vc, const int32_t* src_row, const int32_t* slot, const int32_t* pos, int M,
                  int nlayers, int slots, int Hkv, int S, int HD, hipStream_t st);
// attention.hip
int tb_attention_lds_bytes(int HD);
// decode row count at or below which the 4-wave-per-(row, kv head) decode kernel runs (bit-identical to the one-wave
// kernel), for rows without / with a shared prefix; n < 0: query only; returns the previous value
int tb_attention_split_rows(int n, bool prefix);
// pkc/pvc/pslot/plen (decode only, T == 1; nullptr = none): row b reads keys [0, plen[b]) from slot
// pslot[b] of the shared prefix cache (pkc, pvc) [P, Hkv, S, HD] instead of its own slot.
void tb_attention(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, uint16_t* out, const int32_t* pos,
                  const int32_t* slot, int B, int T, int Hq, int Hkv, int HD, int S, float scale, float softcap,
                  int window, hipStream_t st, const uint16_t* pkc = nullptr, const uint16_t* pvc = nullptr,
                  const int32_t* pslot = nullptr, const int32_t* plen = nullptr);
// blk [nblk, bw]: (first row, rows, slot) (bw = 3) or + (prefix slot, prefix length) (bw = 5, keys below the
// prefix length read from that slot of pkc/pvc).
void tb_attention_varlen(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, uint16_t* out, const int32_t* pos,
                         const int32_t* blk, int nblk, int Hq, int Hkv, int HD, int S, float scale, float softcap,
                         int window, hipStream_t st, int bw = 3, const uint16_t* pkc = nullptr,
                         const uint16_t* pvc = nullptr);
// elementwise.hip
void tb_geglu(const uint16_t* gu, uint16_t* out, int M, int F, hipStream_t st);
// lens.hip
void tb_argmax_rows(const uint16_t* logits, int32_t* out, int R, int V, float cap, hipStream_t st);
void tb_row_lse(const uint16_t* logits, float* lse, int R, int V, float cap, int emulate_bf16, hipStream_t st);
void tb_gather_probs(const uint16_t* logits, const float* lse, const int32_t* ids, float* out, int R, int K, int V,
                     int round_bf16, const int32_t* rowmap, hipStream_t st);
void tb_lens_colsum(const uint16_t* logits, const float* lse, const uint8_t* mask, const int32_t* excl, float* acc,
                    int B, int T, int V, int accumulate, int round_bf16, const int32_t* offs, float* cum,
                    const int32_t* rowmap, hipStream_t st);
// (chunked when C > 1: workspaces wv / wi of R * C * K entries; C from tb_topk_chunks)
int tb_topk_chunks(int R, int V);
void tb_topk_rows(const float* x, float* vals, int32_t* idx, int R, int V, int K, float* wv, int32_t* wi, int C,
                  hipStream_t st);
void tb_xent_rows(const uint16_t* logits, const int32_t* tgt, float* nll, int R, int V, float cap, int emulate_bf16,
                  hipStream_t st);
void tb_register_softcap_table(float cap, const uint16_t* tab);   // [32768] bf16 softcap of +bf16 bit patterns
void tb_decode_head(const uint16_t* logits, const int32_t* tgt, int32_t* nxt, float* nll_self, float* nll_tgt, int R,
                    int V, float cap, hipStream_t st);
// vocab-parallel head: per row {lse, best, best id + off, target logit or -inf} (float4) of this rank's V columns;
// false when the cap has no registered table (caller falls back)
bool tb_decode_head_stats(const uint16_t* logits, const int32_t* tgt, int off, float* stats, int R, int V, float cap,
                          hipStream_t st);
// sae.hip
void tb_head_merge(const float* part, int npart, const int32_t* tgt, const float* tgt_logit, int32_t* nxt,
                   float* nll_self, float* nll_tgt, float* lse, int M, int V, hipStream_t st);
void tb_head_fused4(const uint16_t* A, const uint16_t* W, float* part, float cap, const int32_t* tgt,
                    float* tgt_logit, int32_t* nxt, float* nll_self, float* nll_tgt, int M, int N, int K, hipStream_t st);
// cs: the RoPE table as bf16 (cos, sin) pairs [max_pos, 128, 2] (the fp32 tables rounded once: the epilogue rounds
// them to bf16 anyway, rope.hip's chain)
// a2 / k0 (multi-adapter LoRA): the GEMM's A operand is [A (k0 columns) | a2 (K - k0 columns)] (two sources, no copy)
void tb_gemm4_qkv_rope(const uint16_t* A, const uint16_t* W, const int32_t* pos, const int32_t* slot_of_row,
                       const uint16_t* cs, uint16_t* q_out, uint16_t* kc, uint16_t* vc, int M, int K,
                       int Hq, int Hkv, int S, int max_pos, int tile_rows, hipStream_t st, const uint16_t* a2 = nullptr,
                       int k0 = 0);
bool tb_register_softcap_compact(float cap, const uint16_t* tab, int lo, int hi, float sat);
bool tb_softcap_compact(const uint16_t* x, float* y, int n, float cap, hipStream_t st);
bool tb_gemm4_ok(int M, int N, int K);
int tb_gemm4_splitk_ks(int M, int N, int K, int tile_rows);
int tb_gemm4_splitk_part(const uint16_t* A, const uint16_t* W, float* ws, int M, int N, int K, int tile_rows, int ks,
                         hipStream_t st);
void tb_add_rmsnorm2_part(uint16_t* h, const float* part, int ks, const uint16_t* w_post, const uint16_t* w_next,
                          uint16_t* x, int M, int D, float eps, hipStream_t st);
void tb_gemm4_splitk(const uint16_t* A, const uint16_t* W, uint16_t* out, float* ws, int M, int N, int K, int ldo,
                     int epi, int tile_rows, int ks, hipStream_t st);
// out[b] = sum_t coef[b, t] * (fp32 row at device address ptr[b, t]), V % 4 == 0 (elementwise.hip)
void tb_row_combine(const int64_t* ptr, const float* coef, float* out, int B, int T, int V, hipStream_t st);
bool tb_random_basis_ok(int D);
void tb_random_basis(const uint64_t* seeds, const int32_t* ranks, const int64_t* rows, int n, int D, float* table,
                     hipStream_t st, int qu = 1);
void tb_gemm4(const uint16_t* A, const uint16_t* W, void* C, const float* bias, const float* thr, int M, int N, int K,
              int ldc, int epi, int tile_rows, hipStream_t st, const uint16_t* a2 = nullptr, int k0 = 0);
void tb_gemm_nt(const uint16_t* A, const uint16_t* W, void* C, const float* bias, const float* thr, int M, int N,
                int K, int ldc, int epi, hipStream_t st);
void tb_lowrank_edit(uint16_t* h, uint16_t* x_next, const uint8_t* apply, const int32_t* idx, const int32_t* cnt,
                     int mmax, const void* E, const void* Dm, int table_f32, const float* bias, const float* thr,
                     const float* pre_bias, float alpha, const uint16_t* w_next, float eps, int M, int D,
                     float* coef_out, hipStream_t st);
void tb_sae_decode_sparse(const float* acts, const void* Wdec, int table_f32, const float* b_dec, uint16_t* out_bf16,
                          float* out_f32, int M, int L, int D, hipStream_t st);
void tb_latent_score(const float* acts, const float* p, const uint8_t* spike, const int32_t* seg, float* out,
                     float* spike_mean, float* corr, int G, int L, hipStream_t st);
// p2p.hip
int tb_p2p_header_bytes();
int tb_p2p_max_ranks();
void* tb_p2p_alloc(size_t bytes, int uncached);
int tb_p2p_free(void* p);
int tb_p2p_get_handle(void* p, void* handle_out);
int tb_p2p_handle_size();
void* tb_p2p_open_handle(const void* handle);
int tb_p2p_close_handle(void* p);
int tb_p2p_allreduce(void* const* bases, int rank, int world, const void* in, void* out, size_t nbytes, int is_bf16,
                     int blocks, int spin_max, int barriers, hipStream_t st);
uint32_t tb_p2p_read_error(void* own_base);

// vp.hip: vocab-parallel merges (TP head / lens)
void tb_vp_head_merge(const float* st, int tp, int R, const int32_t* tgt, int V, int32_t* nxt, float* nll_self,
                      float* nll_tgt, hipStream_t stream);
void tb_vp_lse_merge(const float* lse, int tp, int R, float* out, hipStream_t stream);
void tb_vp_topk_merge(const float* vals, const int32_t* ids, int tp, int n, int k, float* ov, int32_t* oi,
                      hipStream_t stream);
int tb_p2p_allgather(void* const* bases, int rank, int world, const void* in, void* out, size_t nbytes, int blocks,
                     int spin_max, int barriers, hipStream_t st);
void tb_slot_copy(uint16_t* dst, const uint16_t* src, const int32_t* dslot, const int32_t* sslot, int n, int nl,
                  int64_t inner, int dst_slots, int src_slots, int dst_l0, int src_l0, hipStream_t st);
void tb_lens_gemm4(const uint16_t* A, const uint16_t* W, uint16_t* logits, float* part, float* lse, int M, int N,
                   int K, hipStream_t st);
// the compact exact softcap registered for `cap` on this device (csrc/lens.hip CapC): table of [lo, hi), saturation
bool tb_softcap_compact_params(float cap, const uint16_t** tab, int* lo, int* hi, float* sat);

// decode_step.hip: per-step bookkeeping of the batched greedy decode (runtime/generation.py)
void tb_decode_pre(const int64_t* step_idx, const int32_t* tf_tgt, int32_t* tf_step, int nb, int W, hipStream_t st);
void tb_decode_post(const int32_t* nxt, const float* nll, const float* tf_nll, uint8_t* done, int64_t* step_idx,
                    int32_t* out_tok, float* out_nll, float* out_tf_nll, const int32_t* stop, int nstop, int32_t* tok,
                    int32_t* pos, int nb, int W, int pad, hipStream_t st);
void tb_share_lo_gather(const int64_t* rep, const int64_t* U, const int32_t* tok, const int32_t* pos,
                        const int32_t* slot, int32_t* s_tok, int32_t* s_pos, int32_t* s_slot, const int32_t* kp_slot,
                        const int32_t* kp_len_lo, int32_t* l_slot, int32_t* l_len_lo, int nb, int B, int S,
                        hipStream_t st);
void tb_capture_rows(uint16_t* store, const uint16_t* h, const int32_t* pos, const int32_t* slot, int n, int T, int S1,
                     int D, hipStream_t st);
void tb_row_gather(uint16_t* out, const uint16_t* src, const void* idx, bool idx64, int n, int D, hipStream_t st);
int tb_share_group_max_rows();
void tb_share_group(int64_t* gid, const int32_t* tok, int64_t* rep, int64_t* grp, int32_t* src, int64_t* U, int nb,
                    int act, int first, int64_t V, hipStream_t st);

// gemm_ring.hip: batch-invariant narrow-tile GEMM (decode / mid row counts); epi 0 bf16, 3 GeGLU (interleaved gate|up)
bool tb_gemm_ring_ok(int M, int N, int K, int epi, int bm, int bn, int var);
int tb_gemm_ring_tiles(int epi, int* bm, int* bn, int cap);
void tb_gemm_ring(const uint16_t* A, const uint16_t* W, uint16_t* C, int M, int N, int K, int ldc, int epi, int bm,
                  int bn, int var, hipStream_t st, const uint16_t* a2 = nullptr, int k0 = 0);
void tb_gemm_ring_qkv_rope(const uint16_t* A, const uint16_t* W, const int32_t* pos, const int32_t* slot_of_row,
                           const uint16_t* cs, uint16_t* q_out, uint16_t* kc, uint16_t* vc, int M,
                           int K, int Hq, int Hkv, int S, int max_pos, int bm, int bn, int var, hipStream_t st,
                           const uint16_t* a2 = nullptr, int k0 = 0);
// multi-adapter LoRA down-projection: T[m, c] = bf16(x[m] . A_all[c]) where column c belongs to the row's adapter
// (c < nsr and (c % nr) / r == adapter[m]), else 0; T is [M, N] (N = A_all rows, the padded LoRA width)
// (K chunked, batch-invariant at every M; part != nullptr: one workgroup per (tile, chunk), fp32 chunk sums in part
// [tb_lora_t_chunks(K), M, N] folded by a second kernel -- the same bits as part == nullptr)
bool tb_lora_t_ok(int M, int N, int K, int bm, int bn);
int tb_lora_t_chunks(int K);
void tb_lora_t(const uint16_t* x, const uint16_t* a_all, uint16_t* t, const int32_t* adapter, int M, int N, int K,
               int nsr, int nr, int r, int bm, int bn, hipStream_t st, int ldt = 0, float* part = nullptr);
