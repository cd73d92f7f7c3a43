// Fused NeRF MLP forward on gfx950 with a 3-term FP16 split of FP32 operands
// (reference src/models/nerf/network.py:49-74, NET): every FP32 product w*x is
// computed as wh*xh + wh*xl + wl*xh on v_mfma_f32_16x16x32_f16 (exact 22-bit
// products, FP32 accumulation), where x = xh + xl, w = wh + wl are the FP16
// round-to-nearest splits of power-of-two-scaled values. 3 MFMAs of 16 cycles
// replace 8 of 32 (FP32 16x16x4) per 16x16x32 tile step: 5.3x the arithmetic
// rate. The dropped wl*xl term and the split residuals are ~2^-22 relative per
// product; scales keep every split in FP16's normal range:
//   * weights: per layer 2^sw (pack time), max |w| * 2^sw in [2^11, 2^12);
//   * activations: per sample and layer 2^e from the sample's max |x| (which
//     includes its encoded input for the skip layer and its view encoding for
//     the views layer), max |x| * 2^e in [2^13, 2^14). A lane holds one sample
//     column of every B operand and accumulator, so the scale is per lane (max
//     over the sample's 4 lane groups: a 2-step butterfly);
//   both undone exactly (power-of-two multiply) before the bias.
//
// Same decomposition and weight streaming as mlp_fused.hip (mlp_stream.h):
// 8 waves x 16 samples, 73 slices of 32 KiB; a slice of a 256-row layer holds
// one 32-deep K step as 16 tiles x (hi, lo) fragment blocks (block 2m + part);
// the views layer packs two K steps per slice (block 16q + 2m + part) and the
// direction step alone in the last slice; the skip layer streams its 8
// activation K steps before its 2 encoding K steps.
//
// Register dataflow: the accumulator of tile m holds, on lane l, sample l&15
// and rows 16m + 4(l>>4) + r. K step q of the next layer takes, on lane group
// g = l>>4, slots j = 0..7 = rows 16(2q + (j>>2)) + 4g + (j&3), i.e. registers
// r of tiles 2q and 2q+1 (nerfhip/pack.py packs W with that K permutation).
// this kernel's weight stream: buffer-form LDS-DMA (mlp_stream.h), issued by
// waves 0-3 only (x3_dma below)
#define MLP_DMA_BUF 1
#include "x3_ops.h"

namespace nerfhip {


// The x3 stream folds the feature layer into the views layer (pack_mlp_x3,
// fold_feature_into_views): 65 slices instead of the FP32 kernel's 73.
constexpr int kX3Slices = NERF_MLP_X3_SLICES;
constexpr int kX3Threads = 64 * kStreamWaves;
constexpr int kX3Tile = 16 * kStreamWaves;

// Cross-slice fragment prefetch: the last group of a slice issues the reads of
// the NEXT slice's group 0 (register set x), so a slice starts its MFMAs right
// after the barrier instead of exposing one LDS latency per slice. The next
// slice must then be visible one barrier earlier: x3_slice_end certifies slice
// g+2 at the end of slice g.

// The fragment register sets, live across slices (x: even groups, y: odd),
// and the stream length (a compile-time constant of each kernel: 65 slices for
// inference and the training forward, where the feature layer is folded into
// the views layer, 64 / 60 for the backward). The backward without the
// encoding products reads the 64-slice stream minus its encoding slices:
// logical slice t >= gap is stored at t + 2 (the last two are never reached;
// nphys slices in memory).
struct FragPipe {
  Frags x, y;
  int ns;
  int gap = 1 << 20;
  int nphys = 0;
};

// The weight stream runs three slices ahead of the compute.
constexpr int kX3DmaAhead = 3;
constexpr int kX3Pieces = 8;   // LDS-DMA pieces per loading wave and slice

// Only waves 0-3 stage weights (8 pieces each, buffer form), so a loading
// wave's SIMD partner (waves 4-7) keeps issuing MFMAs meanwhile (+1.6 %).
// The kernel is persistent (one workgroup per CU loops over sample tiles) and
// the weight stream continues from one tile's last slice into the next tile's
// first, so a tile starts on slices already resident instead of a staged
// prologue. Measured and dropped (round 2): a half-slice stagger of the SIMD
// partners, other loader splits and wave priorities, workgroup start skews.
__device__ __forceinline__ Dma x3_dma(const float4* slices, int t, float* buf, int wave, int lane,
                                      int ns) {
  return make_dma_blocks(slices, t, buf, (wave & 3) * 8, wave, lane, wave < 4, ns);
}

// Group G of NG: drain its fragment reads (issued one group earlier), issue
// group G+1's into the other register set (the last group: the next slice's
// group 0 at LDS base nbase, when NEXT), 6 MFMAs, the wave's LDS-DMA pieces of
// the slice three ahead (after group 0), then the slice's hook for group G:
// VALU work that fills the MFMA shadows (epilogue / operand split, below).
template <int G, int NG, typename Cfg, bool NEXT, typename Acc, typename BV, typename Hook>
__device__ __forceinline__ void run_group3(Acc& acc, unsigned base, unsigned nbase, const BV& bv,
                                           FragPipe& fp, const Dma& dma, Hook& hook) {
  Frags& x = fp.x;
  Frags& y = fp.y;
  if constexpr (G < NG) {
    lds_drain();
    if constexpr (G + 1 < NG) {
      if constexpr ((G & 1) == 0) load_frags<G + 1>(y, base);
      else load_frags<G + 1>(x, base);
    } else if constexpr (NEXT) {
      static_assert((G & 1) == 1, "the last group computes from set y");
      load_frags<0>(x, nbase);
    }
    hook.template prefetch<G>();   // the hook's own LDS reads, drained with the frags
    __builtin_amdgcn_sched_barrier(0);
    constexpr int m = Cfg::tile(G);
    if constexpr ((G & 1) == 0) mfma3x2<Cfg::first(G)>(acc[m], acc[m + 1], x, bv[Cfg::bsel(G)]);
    else mfma3x2<Cfg::first(G)>(acc[m], acc[m + 1], y, bv[Cfg::bsel(G)]);
    // the hook's VALU in the gaps of this group's own MFMAs: MFMA, 2 VALU, ...
    hook.template after<G>(acc);
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // one MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);   // up to 2 VALU
    }
    __builtin_amdgcn_sched_barrier(0);
    // waves 0-3 stage 8 pieces each (after group 0), their partners none
    if constexpr (G == 0) {
      if (dma.live) {
        stage_piece<0>(dma); stage_piece<1>(dma); stage_piece<2>(dma); stage_piece<3>(dma);
        stage_piece<4>(dma); stage_piece<5>(dma); stage_piece<6>(dma); stage_piece<7>(dma);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    run_group3<G + 1, NG, Cfg, NEXT>(acc, base, nbase, bv, fp, dma, hook);
  }
}

// Slice g of the stream (NG groups). Its group 0 fragments were issued by the
// previous slice's last group (or the kernel prologue).
template <int NG, typename Cfg, bool NEXT = true, typename Acc, typename BV, typename Hook>
__device__ __forceinline__ void run_slice3(Acc& acc, const Ring& R, int g, const BV& bv,
                                           FragPipe& fp, Hook& hook) {
  const unsigned base = lds_base(R.buf(g), R.lane);
  const int t = g + kX3DmaAhead;
  // the stream runs on into the next tile (the last tile's wrapped pieces are
  // staged but never read): every slice stages one, every slice_end counts 2
  int ts = t < fp.ns ? t : t - fp.ns;
  ts += ts >= fp.gap ? 2 : 0;
  run_group3<0, NG, Cfg, NEXT>(acc, base, lds_base(R.buf(g + 1), R.lane), bv, fp,
                               x3_dma(R.slices, ts, R.buf(t), R.wave, R.lane,
                                      fp.nphys ? fp.nphys : fp.ns), hook);
}

// End of slice g: this wave's LDS-DMA of slice g+2 has landed (the next
// slice's group 0 fragments are read before this barrier), then one barrier
// publishes it to every wave and frees slice g's buffer for the DMA issued in
// slice g+1. INFLIGHT = slices of DMA that could stay in flight without that
// prefetch (2 while the stream has three slices ahead).
template <int INFLIGHT>
__device__ __forceinline__ void x3_slice_end(const FragPipe&) {
  slice_end<(INFLIGHT > 0 ? INFLIGHT - 1 : 0), kX3Pieces>();
}



struct NoHook {
  template <int G>
  __device__ __forceinline__ void prefetch() {}
  template <int G, typename Acc>
  __device__ __forceinline__ void after(Acc&) {}
};

// Splits operand `op` (FP32 -> FP16 hi/lo at scale s) across the slice's even
// groups: values 2k, 2k+1 after group 2k into a temporary, committed after the
// last group (the operand is not read by this slice).
// The empty asm takes the results as register operands at this point of the
// program, so IR-level sinking cannot move the work to the commit.
struct SplitHook {
  Op& op;
  float s;
  Op t;
  template <int G>
  __device__ __forceinline__ void prefetch() {}
  template <int G, typename Acc>
  __device__ __forceinline__ void after(Acc&) {
    if constexpr ((G & 1) == 0 && G < 8) {
      float hp, lp;
      split2(op[G], op[G + 1], s, hp, lp);
      asm volatile("" : "+v"(hp), "+v"(lp));
      t[G / 2] = hp;
      t[4 + G / 2] = lp;
    }
    if constexpr (G == 7) op = t;
  }
};

// TRAIN: an operand pair of the previous layer's output (FP32, before its split)
// is written to HBM at the start of the slice that splits it -- before the
// slice issues its LDS-DMA pieces, so the slice's closing counted vmcnt (which
// lets the pieces stay in flight) only waits for stores issued a slice
// earlier. Stores issued after the pieces would make that wait drain the
// pieces (vmcnt counts loads, stores and LDS-DMA together, in issue order).
// NoPend: inference (nothing stored).
struct NoPend {
  template <int P>
  __device__ __forceinline__ void pair(const Op&) {}
  template <int P, int R>
  __device__ __forceinline__ void part(const Op&) {}
};

// NERF_STORE_SPREAD (a study build, never shipped; round 4's store-spreading
// variant recreated for the static ISA check): the waves that stage
// no weight pieces (4-7) spread a pair's stores over groups 0-3, two per group
#ifndef NERF_STORE_SPREAD
#define NERF_STORE_SPREAD 0
#endif
#ifndef NERF_ABL_NOSTORE
#define NERF_ABL_NOSTORE 0
#endif
template <int P, int G, typename Pend>
__device__ __forceinline__ void store_pair_at(Pend& st, const Op& v) {
#if NERF_STORE_SPREAD
  const bool loader = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) < 4;
  if (loader) {
    if constexpr (G == 0) st.template pair<P>(v);
  } else if constexpr (G < 4) {
    st.template part<P, G>(v);
  }
#else
  if constexpr (G == 0) st.template pair<P>(v);
#endif
}

template <int P, typename Pend, typename Split>
struct StoreThen {
  Pend& st;
  Split sp;
  template <int G>
  __device__ __forceinline__ void prefetch() {}
  template <int G, typename Acc>
  __device__ __forceinline__ void after(Acc& acc) {
    // behind group 0's MFMAs (they issue first), ahead of the slice's pieces
    store_pair_at<P, G>(st, sp.op);
    sp.template after<G>(acc);
  }
};

// two operand splits in one slice (views layer)
struct Split2 {
  SplitHook a, b;
  template <int G>
  __device__ __forceinline__ void prefetch() {}
  template <int G, typename Acc>
  __device__ __forceinline__ void after(Acc& acc) {
    a.template after<G>(acc);
    b.template after<G>(acc);
  }
};

template <int P, typename Pend>
struct StoreThen2 {   // views slice: pairs P, P+1 stored, then split
  Pend& st;
  Split2 sp;
  template <int G>
  __device__ __forceinline__ void prefetch() {}
  template <int G, typename Acc>
  __device__ __forceinline__ void after(Acc& acc) {
    if constexpr (G == 0) {   // behind group 0's MFMAs, ahead of the slice's pieces
      st.template pair<P>(sp.a.op);
      st.template pair<P + 1>(sp.b.op);
    }
    sp.template after<G>(acc);
  }
};

// Epilogue of a 256-row layer fused into its last slice (the K step that reads
// operand 7 only): after group G, tiles 2G, 2G+1 are final -> acc * 2^-shift +
// bias, ReLU floor, into operand X[G] as FP32 (split later); running |max|;
// density-head partial dot (layer 7). The next layer's first slice restarts the
// accumulators from zero.
// The power-of-two product is exact, so the fma rounds like the reference's add.
struct EpiHook {
  Op (&X)[8];
  float inv, floor;
  unsigned bias;       // LDS byte address of this lane group's packed biases [4m + r]
  const float* aw;     // density-head weights (layer 7) or nullptr
  float amax, apart;
  bool on;             // false: the layer continues after this slice
  f32x4 bb[2][2];      // biases of pairs G (G & 1), loaded in group G's read phase
  template <int G>
  __device__ __forceinline__ void prefetch() {
    if constexpr (G < 8) {
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bb[G & 1][0]) : "v"(bias), "i"(32 * G) : "memory");
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bb[G & 1][1]) : "v"(bias), "i"(32 * G + 16) : "memory");
    }
  }
  // in the slice: tile pair G-1 after group G (its MFMA results have landed
  // while group G issued); pair 7 by finish() after the slice
  template <int G, typename Acc>
  __device__ __forceinline__ void after(Acc& acc) {
    if constexpr (G >= 1 && G <= 8) pair<G - 1>(acc);
  }
  template <typename Acc>
  __device__ __forceinline__ void finish(Acc& acc) {
    lds_drain();   // pair 7's biases (read in group 7)
    pair<7>(acc);
  }
  template <int G, typename Acc>
  __device__ __forceinline__ void pair(Acc& acc) {
    {
      if (!on) return;
      Op v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = fmaxf(__builtin_fmaf(acc[2 * G][r], inv, bb[G & 1][0][r]), floor);
        v[4 + r] = fmaxf(__builtin_fmaf(acc[2 * G + 1][r], inv, bb[G & 1][1][r]), floor);
      }
#pragma unroll
      for (int j = 0; j < 8; j += 2)
        asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(amax) : "v"(v[j]), "v"(v[j + 1]));
      if (aw) {
#pragma unroll
        for (int j = 0; j < 8; ++j) apart = __builtin_fmaf(v[j], aw[8 * G + j], apart);
      }
      asm volatile("" : "+v"(v), "+v"(amax));   // computed here, not sunk to the use
      X[G] = v;
    }
  }
};


// One 256-row slice (K step Q of operand array B) + its end-of-slice sync.
template <int Q, bool FIRST, typename BV, typename Hook>
__device__ __forceinline__ void slice256x(f32x4 (&acc)[16], const Ring& R, int g, const BV& b,
                                          FragPipe& fp, Hook& hook) {
  run_slice3<8, Step256<Q, FIRST>>(acc, R, g, b, fp, hook);
  x3_slice_end<2>(fp);
}
template <int Q, typename BV, typename Hook>
__device__ __forceinline__ void slice256(f32x4 (&acc)[16], const Ring& R, int g, const BV& b,
                                         FragPipe& fp, Hook& hook) {
  slice256x<Q, false>(acc, R, g, b, fp, hook);
}

// A whole epilogue outside a slice (skip layer): each pair's biases, then it.
template <int P, typename Epi>
__device__ __forceinline__ void epi_pairs(Epi& epi, f32x4 (&acc)[16]) {
  if constexpr (P < 8) {
    epi.template prefetch<P>();
    lds_drain();
    epi.template pair<P>(acc);
    epi_pairs<P + 1>(epi, acc);
  }
}

// The 8 activation slices g .. g+7 of a layer: the first restarts the
// accumulators, slice q splits operand q+1 (scale s) in its MFMA shadows, the
// last runs the fused epilogue (disabled for the skip layer, whose two
// encoding slices follow).
template <typename Epi, typename Pend>
__device__ __forceinline__ void act_slices(f32x4 (&acc)[16], const Ring& R, int g, Op (&X)[8],
                                           float s, FragPipe& fp, Epi& epi, Pend& st) {
  { StoreThen<1, Pend, SplitHook> h{st, {X[1], s}}; slice256x<0, true>(acc, R, g + 0, X, fp, h); }
  { StoreThen<2, Pend, SplitHook> h{st, {X[2], s}}; slice256<1>(acc, R, g + 1, X, fp, h); }
  { StoreThen<3, Pend, SplitHook> h{st, {X[3], s}}; slice256<2>(acc, R, g + 2, X, fp, h); }
  { StoreThen<4, Pend, SplitHook> h{st, {X[4], s}}; slice256<3>(acc, R, g + 3, X, fp, h); }
  { StoreThen<5, Pend, SplitHook> h{st, {X[5], s}}; slice256<4>(acc, R, g + 4, X, fp, h); }
  { StoreThen<6, Pend, SplitHook> h{st, {X[6], s}}; slice256<5>(acc, R, g + 5, X, fp, h); }
  { StoreThen<7, Pend, SplitHook> h{st, {X[7], s}}; slice256<6>(acc, R, g + 6, X, fp, h); }
  slice256<7>(acc, R, g + 7, X, fp, epi);
  epi.finish(acc);
}

// ---------------------------------------------------------------------------
// The training forward (TRAIN): the same kernel over the same 65-slice stream
// (round 5: the feature layer folded into the views layer from the step's own
// parameters by nerf_fold_views; the feature rows are never formed, the
// views / feature weight gradients go through h7), which also writes every
// layer's output FP32 rows to HBM feature-
// major ([F][P], row stride ld: what the backward's weight gradients read),
// the ReLU bits of h0..h7 and of the views layer in x3_layer_kernel's mask-bit
// layout (its dgrad launches read them), and each output's max |.| (the weight
// gradients' FP16 scales) -- one launch instead of ten x3_layer_kernel
// launches, the activations never read back from HBM.
// ---------------------------------------------------------------------------
// LDS atomic max (the outputs' max |.|: non-negative floats compare as their
// bits) as inline asm: hipcc places an s_waitcnt vmcnt(0) before any compiler-
// visible DS instruction while LDS-DMA may be in flight (it cannot prove the
// addresses apart), which would drain the weight stream's pieces and the
// activation stores at every layer. Completed by the next lgkmcnt(0) drain.
__device__ __forceinline__ void lds_max_u32(unsigned* p, unsigned v) {
  asm volatile("ds_max_u32 %0, %1" ::"v"(lds_addr(reinterpret_cast<const float*>(p))), "v"(v)
               : "memory");
}

// cache policy of the training kernels' activation / gradient row stores
// (buffer instruction aux bits): nt (2). The rows are read back by another
// kernel after gigabytes of other traffic, never from L2; the weight stream the
// same kernels read is. C3 3.50 vs 3.56 ms with the default policy, sc1 (16)
// 3.67 (tools/gpu_ab_wgrad.sh, two interleaved runs each; `make variant`)
#ifndef NERF_ACT_STORE_AUX
#define NERF_ACT_STORE_AUX 2
#endif

// Where element (row, sample p) of a training activation / gradient buffer
// lives, in floats from the output's pointer (rows start on 16-row groups).
// bs == 0: feature-major rows [rows][ld], element row * ld + p. bs > 0: the
// 16-sample tile layout T16 -- a block of 16 samples holds every row of the
// buffer (block stride bs floats), and inside it each 16-row group is one
// 1-KiB tile with row 16 t + 4 g + r of sample s at t * 256 + r * 64 + g * 16 + s.
// Element r of a 16 x 16 MFMA accumulator tile (lane 16 g + s holds rows 4 g ..
// 4 g + 3 of sample s) is then 256 contiguous bytes for the whole wave: one
// store instruction writes whole lines, and a K step of the weight gradients
// (32 samples) reads two contiguous 16-KiB runs per 256-row operand
// (NerfWgradDesc bsa / bsb; nerfhip.train_mlp.BlockRows).
struct Lay {
  int64_t ld, bs;
  int64_t nblk;   // T16: the buffer's 16-sample blocks (whole 128-sample tiles)
  __device__ __forceinline__ static int rowpart(int row) {   // T16, floats
    return (row >> 4) * 256 + (row & 3) * 64 + ((row >> 2) & 3) * 16;
  }
  // element (row, p), bytes (T: the T16 layout, a kernel's compile-time choice)
  template <bool T>
  __device__ __forceinline__ unsigned elem(int row, int64_t p) const {
    if constexpr (T) return (unsigned)(((p >> 4) * bs + rowpart(row) + (p & 15)) * 4);
    else return (unsigned)(((int64_t)row * ld + p) * 4);
  }
  // bytes an output of `rows` rows spans from its pointer (its num_records)
  template <bool T>
  __device__ __forceinline__ int extent(int rows) const {
    if constexpr (T) return (int)(((nblk - 1) * bs + ((rows + 15) & ~15) * 16) * 4);
    else return (int)((int64_t)rows * ld * 4);
  }
};

// The head block's LDS image in the x3 kernels: the global layout (mlp_stream.h)
// with the biases [9][4][64] and the density-head weights [4][64] padded to 68
// floats per lane group. A ds_read_b128 serves its lanes in four 16-lane groups
// (lanes 0-3, 12-15, 20-27, ...: MI355X_MICROARCH.md LDS), which mix lane groups
// g4 0 and 1 (2 and 3); their bias vectors 64 floats apart share banks (a
// 2-way conflict on every epilogue bias read: SQ_LDS_BANK_CONFLICT ~640 cycles
// per wave and tile), 68 floats apart they do not.
constexpr int kLdsGroup = 68;                              // floats per lane group
constexpr int kLdsBias = 0;                                // [9][4][68]
constexpr int kLdsBiasViews = 9 * 4 * kLdsGroup;           // [4][32]
constexpr int kLdsAlphaW = kLdsBiasViews + 128;            // [4][68]
constexpr int kLdsTail = kLdsAlphaW + 4 * kLdsGroup;       // kHeadAlphaB .. the end, shifted
constexpr int kHeadLds = kLdsTail + (kHeadFloats - kHeadAlphaB);
static_assert(kHeadBiasViews == 9 * 256 && kHeadAlphaW == kHeadBiasViews + 128 &&
                  kHeadAlphaB == kHeadAlphaW + 256 && kLdsAlphaW % 4 == 0 && kLdsTail % 4 == 0,
              "head layout (mlp_stream.h) and its LDS image disagree");
// LDS float index of head float f (f % 4 == 0 keeps a float4 together)
__host__ __device__ constexpr int head_lds(int f) {
  return f < kHeadBiasViews ? (f / 256) * 4 * kLdsGroup + (f % 256 / 64) * kLdsGroup + f % 64
       : f < kHeadAlphaW    ? kLdsBiasViews + (f - kHeadBiasViews)
       : f < kHeadAlphaB    ? kLdsAlphaW + (f - kHeadAlphaW) / 64 * kLdsGroup + (f - kHeadAlphaW) % 64
                            : kLdsTail + (f - kHeadAlphaB);
}
// the head block (global) into its LDS image, float4 by float4
__device__ __forceinline__ void load_head_lds(float* hd, const float* head, int tid, int nthreads) {
  for (int i = tid; i < kHeadFloats / 4; i += nthreads)
    *reinterpret_cast<float4*>(hd + head_lds(4 * i)) = reinterpret_cast<const float4*>(head)[i];
}

struct ActStore {
  __amdgpu_buffer_rsrc_t rs;   // the layer's output rows (num_records: Lay::extent)
  __amdgpu_buffer_rsrc_t rb;   // its ReLU-bit words (num_records 0: no bits)
  unsigned soff;               // uniform: this (tile, wave)'s first sample / block, bytes
  unsigned sboff;              // uniform: this (tile, wave)'s first bit word, * 2
  unsigned c4, ts, rstr;       // uniform, bytes: per lane group g4 (rows 4 g4 ..), per
                               // 16-row tile, per row r of a lane's 4 (Lay; set by set_lay)
  unsigned wb;                 // bits of the current 4-tile block
  bool bits, valid;
  bool on = true;              // uniform: false = these rows are not stored (null output)
  __device__ __forceinline__ void st32(float x, unsigned vo, int off) const {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), rs, (int)vo, off, NERF_ACT_STORE_AUX);
  }
  template <bool T>
  __device__ __forceinline__ void set_lay(const Lay& L, int64_t tile, int wave) {
    if constexpr (T) {
      soff = (unsigned)((tile * 8 + wave) * L.bs * 4);
      c4 = 64u; ts = 1024u; rstr = 256u;
    } else {
      soff = (unsigned)((tile * kX3Tile + wave * 16) * 4);
      c4 = (unsigned)(L.ld * 16); ts = (unsigned)(L.ld * 64); rstr = (unsigned)(L.ld * 4);
    }
  }
  // this lane's offset of its rows 4 g4 + r of tile t: lane_off() + t * ts + r * rstr
  __device__ __forceinline__ unsigned lane_off() const {
    unsigned lid = __lane_id();
    asm volatile("" : "+v"(lid));
    return valid ? (lid >> 4) * c4 + (lid & 15u) * 4u + soff : 0x7fffffffu;
  }
  // (NERF_STORE_SPREAD study builds) element R of pair G's two tiles; the bits
  // of the pair with its last element
  template <int G, int R>
  __device__ __forceinline__ void part(const Op& v) {
    if (!on) return;
    const unsigned vo = lane_off();
    st32(v[R], vo, (int)(2 * G * ts + R * rstr));
    st32(v[4 + R], vo, (int)((2 * G + 1) * ts + R * rstr));
    if constexpr (R == 3) store_bits<G>(v);
  }
  template <int G>
  __device__ __forceinline__ void store_bits(const Op& v) {
    if (bits) {   // bit 4t + r of the block word = (h > 0): post-ReLU h >= 0
      unsigned m = 0u;
#pragma unroll
      for (int j = 0; j < 8; ++j) m |= min(__float_as_uint(v[j]), 1u) << j;
      if constexpr ((G & 1) == 0) {
        wb = m;
      } else {
        wb |= m << 8;
        if (valid)
          __builtin_amdgcn_raw_buffer_store_b16((unsigned short)wb, rb, (int)(__lane_id() * 2u),
                                                (int)(sboff + (G >> 1) * 128), 0);
      }
    }
  }
  // pair G = tiles 2G (v[0..3], rows 32G + 4 g4 + r) and 2G+1 (v[4..7], rows + 16).
  // The lane's offsets are recomputed here (a few VALU in the MFMA shadows)
  // instead of living in VGPRs through the whole tile.
  template <int G>
  __device__ __forceinline__ void pair(const Op& v) {
    if (!on) return;
#if NERF_ABL_NOSTORE == 1   // timing-only ablation build: no row / bit stores (wrong results)
    asm volatile("" ::"v"(v));
    return;
#elif NERF_ABL_NOSTORE == 2   // timing-only: the stores issued, all dropped by the range check
    rs = __builtin_amdgcn_make_buffer_rsrc((void*)nullptr, 0, 0, 0x00020000);
    rb = rs;
#endif
    const unsigned vo = lane_off();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#if NERF_ABL_NOSTORE == 3   // timing-only: half the row stores issued (wrong results)
      if (r >= 2) continue;
#endif
      st32(v[r], vo, (int)(2 * G * ts + r * rstr));
      st32(v[4 + r], vo, (int)((2 * G + 1) * ts + r * rstr));
    }
    store_bits<G>(v);
  }
};

// Output locations of the training forward (nerf_mlp_train_forward_x3).
struct X3TrainOut {
  float* act[12];               // h0..h7, feature, views-layer output, the xyz encoding (64
                                // rows, 63 = 0), the view encoding (32 rows, 27.. = 0); stride ld
  unsigned short* bits[9];      // ReLU bits of h0..h7 (x3_layer_kernel MT 16) and views (MT 8)
  float* amax;                  // [12]: raised to max |.| of h0..h7 (0-7), feature (8), xyz
                                // encoding (9), view encoding (10), views (11)
  Lay lay;                      // every output's layout (row stride / T16 block stride)
};

// Encoding rows of the training forward: the feature index (freq.py's column
// order) of slot (q, j) of lane group g in encode_xyz's register layout
// (x3_cols_enc), 63 for its one padding slot; encode_dir's (x3_cols_dir), 27..31
// for its padding slots. Every row 0..63 / 0..31 is written exactly once.
__device__ __forceinline__ int enc_xyz_row(int g, int q, int j) {
  const int t = 4 * q + (j >> 1), pr = 8 * g + t;
  if (pr < 30) return ((j & 1) ? 6 : 3) + 6 * (pr / 3) + pr % 3;
  return t == 6 ? (j & 1) : ((j & 1) ? 63 : 2);
}
__device__ __forceinline__ int enc_dir_row(int g, int j) {
  if (j < 6) return ((j & 1) ? 6 : 3) + 6 * g + (j >> 1);
  if (j == 6) return g < 3 ? g : 27;
  return 28 + g;
}

// The range check of a raw buffer access covers voffset + soffset + the
// instruction offset, and drops an access that straddles num_records
// (tools/probe/buffer_range.hip on gfx950). So the samples past P are dropped by
// voffset 0x7fffffff whatever row offset rides in soffset (rows * ld * 4 < 2^31
// is enforced by the launchers: the sum cannot wrap), and a null output (the
// skipped feature / DF rows) gets num_records 0: every store through it is
// dropped even if a path forgets the ActStore::on test.
template <bool T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(float* p, int rows, const Lay& L) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, p ? L.template extent<T>(rows) : 0,
                                           0x00020000);
}

// LIST: the samples are the flat indices list[0 .. *count) (ray * S + step,
// written by the ERT segment kernel; the count is read on the device, so a
// segmented evaluation needs no host round trip); raw is written at those
// indices. Otherwise the samples are 0 .. total.
// TRACE (diagnostic twin only): the first lane of workgroups 0..3 stamps
// s_memtime at each of its first 32 tiles' start, after the tile's sample
// loads + encoding, and at its end: trace[(b * 32 + i) * 4 + 0..2]; [3]: after
// the loads, before the encoding.
template <bool LIST, bool TRAIN, bool TRACE = false, bool T16 = false>
__device__ __forceinline__ void mlp_x3_body(
    const float4* __restrict__ slices, const float* __restrict__ head,
    const float* __restrict__ rays_o, const float* __restrict__ rays_d,
    const float* __restrict__ z, int64_t z_stride, int64_t total, int S,
    float4* __restrict__ raw, const int* __restrict__ list, const int* __restrict__ count,
    const X3TrainOut& to, unsigned long long* trace = nullptr) {
  if constexpr (LIST) total = *count;
  __shared__ __attribute__((aligned(16))) float ring[4 * kSliceFloats];
  __shared__ __attribute__((aligned(16))) float hd[kHeadLds];
  __shared__ unsigned amax_lds[12];   // TRAIN: this workgroup's max |.| per output

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  Ring R{ring, slices, wave, lane};
  constexpr int kNs = kX3Slices;   // TRAIN too: the feature layer folded (round 5)

  for (int t = 0; t < kX3DmaAhead; ++t)   // all 8 waves, 4 pieces each
    stage_slice(TRAIN ? make_dma_blocks(slices, t, R.buf(t), wave * kBlocksPerWave, wave, lane,
                                        true, kNs)
                      : make_dma(slices, t, R.buf(t), wave, lane));
  load_head_lds(hd, head, tid, kX3Threads);
  if constexpr (TRAIN) {
    if (tid < 12) amax_lds[tid] = 0u;
  }

  FragPipe fp;
  fp.ns = kNs;
  const int64_t ntiles = (total + kX3Tile - 1) / kX3Tile;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
  const bool first_tile = tile == (int64_t)blockIdx.x;
  const int64_t gs = tile * kX3Tile + wave * 16 + (lane & 15);
  const int ti = (int)((tile - blockIdx.x) / gridDim.x);
  const bool tr = TRACE && blockIdx.x < 4 && ti < 32 && threadIdx.x == 0;
  unsigned long long* trp = TRACE ? trace + ((int64_t)blockIdx.x * 32 + ti) * 4 : nullptr;
  if constexpr (TRACE) {
    if (tr) trp[0] = __builtin_amdgcn_s_memtime();
  }
  // recomputed per tile: otherwise the encoding's per-lane constants are
  // hoisted out of the tile loop and, live through every slice, spill
  int g4 = lane >> 4;
  asm volatile("" : "+v"(g4));
  const bool valid = gs < total;
  const int64_t gl = valid ? gs : total - 1;
  const int64_t gc = LIST ? (int64_t)list[gl] : gl;   // the flat sample index
  const int64_t ray = gc / S;
  const int step = (int)(gc - ray * S);
  const float zv = z[ray * z_stride + step];
  float p[3], dv[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    dv[c] = rays_d[ray * 3 + c];
    p[c] = rays_o[ray * 3 + c] + dv[c] * zv;      // VR:165: o + d*z, two roundings
  }
  if constexpr (TRACE) {   // the sample inputs have landed (before the encoding)
    asm volatile("" ::"v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(dv[0]), "v"(dv[1]), "v"(dv[2]));
    if (tr) trp[3] = __builtin_amdgcn_s_memtime();
  }
  Op encf[2];                   // FP32 encoding (split in place for the skip layer)
  encode_xyz(p, g4, encf);
  const float enc_max = sample_max(fmaxf(op_absmax(encf[0]), op_absmax(encf[1])));
  if constexpr (TRACE) {
    asm volatile("" ::"v"(enc_max));
    if (tr) trp[1] = __builtin_amdgcn_s_memtime();
  }
  if constexpr (TRAIN) {   // the encoding rows (the wgrad operand of layers 0 and 5)
    int i10 = 10;
    asm volatile("" : "+s"(i10));
    const __amdgpu_buffer_rsrc_t rs = rows_rsrc<T16>(to.act[i10], 64, to.lay);
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned vo = valid ? to.lay.template elem<T16>(enc_xyz_row(g4, q, j), gs)
                                  : 0x7fffffffu;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(encf[q][j]), rs, (int)vo, 0, 0);
      }
  }

  using Epi = EpiHook;   // (the training stores ride on the next slices' hooks)
  using Pend = typename std::conditional<TRAIN, ActStore, NoPend>::type;
  // TRAIN: where this (tile, wave) writes (uniform parts; the lane's own part is
  // recomputed at each store)
  auto store_for = [&](int L, int rows) {
    Pend st;
    if constexpr (TRAIN) {
      const int wv = __builtin_amdgcn_readfirstlane(wave);
      // the layer's pointers are loaded from the kernel arguments here, at the
      // layer (an opaque index: kept live through the whole tile loop, the 19
      // pointers would not fit the SGPR budget)
      int Li = L;
      asm volatile("" : "+s"(Li));
      st.rs = rows_rsrc<T16>(to.act[Li], rows, to.lay);
      st.on = to.act[Li] != nullptr;   // the feature rows may be skipped (act[8] null)
      st.bits = L < 8;
      st.rb = __builtin_amdgcn_make_buffer_rsrc((void*)to.bits[Li < 8 ? Li : 0], 0,
                                                L < 8 ? 0x7fffffff : 0, 0x00020000);
      st.template set_lay<T16>(to.lay, tile, wv);
      st.sboff = (unsigned)(((tile * 8 + wv) * 4) * 64 * 2);
      st.wb = 0u;
      st.valid = valid;
    } else {
      (void)L;
      (void)rows;
    }
    return st;
  };
  auto amax_to_lds = [&](int slot, float mx) {
    if constexpr (TRAIN) lds_max_u32(&amax_lds[slot], __float_as_uint(mx));
  };

  f32x4 acc[16];   // every layer's first slice starts it from zero
  Op X[8];
  if (first_tile) __syncthreads();   // head, z/rays loads and the three prologue slices resident
  // slice 0, group 0 (a later tile's slice 0 was certified by the previous
  // tile's slice 63; not prefetched across tiles: the fragments would stay live
  // through the tail and the encoding)
  load_frags<0>(fp.x, lds_base(R.buf(0), lane));

  // ---- layer 0: 63 -> 256 (slices 0, 1), epilogue fused into slice 1 --------
  int e = act_exponent(enc_max);
  float s = ldexpf(1.0f, e);
  {
    Op E[2] = {encf[0], encf[1]};   // split copy: the FP32 encoding returns at layer 5
    split_op(E[0], s);
    split_op(E[1], s);
    NoHook nh;
    slice256x<0, true>(acc, R, 0, E, fp, nh);
    Epi epi{X, ldexpf(1.0f, -((int)hd[head_lds(kHeadScales) + 0] + e)), 0.0f,
            lds_addr(hd + kLdsBias + g4 * kLdsGroup), nullptr, 0.0f, 0.0f, true};
    slice256<1>(acc, R, 1, E, fp, epi);
    epi.finish(acc);
    amax_to_lds(0, epi.amax);
    amax_to_lds(9, enc_max);
    e = act_exponent(sample_max(epi.amax));
  }
  // TRAIN: h0 goes to HBM pair by pair in the next layer's slices (pair 0 now)
  Pend st = store_for(0, 256);
  st.template pair<0>(X[0]);
  s = ldexpf(1.0f, e);
  split_op(X[0], s);
  int g = 2;

  float alpha = 0.0f;
  float mx7 = 0.0f;
  // ---- layers 1..7 (skip input at 5) ------------------------------------------
  // (inference: the feature layer, NET:63, has no activation, and pack_mlp_x3
  // folds it into the views layer, which then reads h7 directly)
  for (int L = 1; L <= 7; ++L) {
    Epi epi{X, ldexpf(1.0f, -((int)hd[head_lds(kHeadScales) + L] + e)), 0.0f,
            lds_addr(hd + kLdsBias + L * 4 * kLdsGroup + g4 * kLdsGroup),
            L == 7 ? hd + kLdsAlphaW + g4 * kLdsGroup : nullptr, 0.0f, 0.0f, L != 5};
    act_slices(acc, R, g, X, s, fp, epi, st);   // stores h_{L-1} pairs 1..7
    g += 8;
    if (L == 5) {   // cat(input_pts, h) (NET:57-58): the encoding's K steps last
      NoHook nh;
      slice256<0>(acc, R, g, encf, fp, nh);
      slice256<1>(acc, R, g + 1, encf, fp, nh);
      g += 2;
      epi.on = true;   // this layer's epilogue, not pipelined
      epi_pairs<0>(epi, acc);
    }
    amax_to_lds(L, epi.amax);
    if (L == 7) alpha = quad_sum(epi.apart) + hd[head_lds(kHeadAlphaB)];   // NET:61
    // the next layer's input scale (the skip layer's covers the encoding too)
    float mx = epi.amax;
    if (L == 4) mx = fmaxf(mx, enc_max);
    st = store_for(L, 256);
    st.template pair<0>(X[0]);
    if (L == 7) {
      mx7 = mx;
      break;
    }
    e = act_exponent(sample_max(mx));
    s = ldexpf(1.0f, e);
    split_op(X[0], s);
    if (L == 4) {   // the FP32 encoding is not needed after the skip layer
      split_op(encf[0], s);
      split_op(encf[1], s);
    }
  }
  // acc holds zeros; X holds h7 (FP32, unsplit)
  if constexpr (TRAIN) {   // h7 pair 1 now; pairs 2..7 ride on the views slices' hooks
    st.template pair<1>(X[1]);
  }
  (void)mx7;

  // ---- views layer: cat(feature, input_views) 283 -> 128, ReLU (NET:62-67),
  // feature = W_f h7 + b_f folded in (W_views,feat W_f on h7; training: the
  // per-step fold of nerf_fold_views) ---------------------------------------------
  Op dirf;
  encode_dir(dv, g4, dirf);
  if constexpr (TRAIN) {   // the view-encoding rows (the views layer's wgrad operand)
    int i11 = 11;
    asm volatile("" : "+s"(i11));
    const __amdgpu_buffer_rsrc_t rs = rows_rsrc<T16>(to.act[i11], 32, to.lay);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned vo = valid ? to.lay.template elem<T16>(enc_dir_row(g4, j), gs) : 0x7fffffffu;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dirf[j]), rs, (int)vo, 0, 0);
    }
    amax_to_lds(10, op_absmax(dirf));
  }
  {
    float mx = op_absmax(dirf);
#pragma unroll
    for (int q = 0; q < 8; ++q) mx = fmaxf(mx, op_absmax(X[q]));
    e = act_exponent(sample_max(mx));
  }
  s = ldexpf(1.0f, e);
  split_op(X[0], s);
  split_op(X[1], s);
  f32x4 acc8[8];   // started from zero by the first views slice
  {
    // views slice k reads operands 2k, 2k+1 and splits 2k+2, 2k+3 (then dir)
    StoreThen2<2, Pend> h0{st, {{X[2], s}, {X[3], s}}};
    run_slice3<8, StepViews<0, true>>(acc8, R, g, X, fp, h0); x3_slice_end<2>(fp);
    StoreThen2<4, Pend> h1{st, {{X[4], s}, {X[5], s}}};
    run_slice3<8, StepViews<2>>(acc8, R, g + 1, X, fp, h1); x3_slice_end<2>(fp);
    StoreThen2<6, Pend> h2{st, {{X[6], s}, {X[7], s}}};
    run_slice3<8, StepViews<4>>(acc8, R, g + 2, X, fp, h2); x3_slice_end<2>(fp);
    SplitHook h3{dirf, s};
    run_slice3<8, StepViews<6>>(acc8, R, g + 3, X, fp, h3); x3_slice_end<2>(fp);
    NoHook nh;
    const Op D[1] = {dirf};
    run_slice3<4, Step256<0>, false>(acc8, R, g + 4, D, fp, nh); x3_slice_end<2>(fp);
  }
  {   // views epilogue (bias, ReLU) -- once per pass, not pipelined
    const float inv = ldexpf(1.0f, -((int)hd[head_lds(kHeadScales) + 9] + e));
    const float* bias = hd + kLdsBiasViews + g4 * 32;
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        acc8[m][r] = fmaxf(__builtin_fmaf(acc8[m][r], inv, bias[4 * m + r]), 0.0f);
  }
  if constexpr (TRAIN) {   // the views output rows, its ReLU bits (MT 8) and max
    int i9 = 9;
    asm volatile("" : "+s"(i9));
    const __amdgpu_buffer_rsrc_t rs = rows_rsrc<T16>(to.act[i9], 128, to.lay);
    ActStore sv;
    sv.valid = valid;
    sv.template set_lay<T16>(to.lay, tile, wave);
    const unsigned voff = sv.lane_off();
    float vmax = 0.0f;
#pragma unroll
    for (int u0 = 0; u0 < 8; u0 += 4) {
      unsigned wb = 0u;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc8[u0 + t][r];
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, (int)voff,
                                                (int)((u0 + t) * sv.ts + r * sv.rstr), 0);
          wb |= min(__float_as_uint(v), 1u) << (4 * t + r);
          vmax = fmaxf(vmax, v);
        }
      if (valid) to.bits[i9 - 1][(((tile * 8 + wave) * 8 + u0) / 4) * 64 + lane] = (unsigned short)wb;
    }
    amax_to_lds(11, vmax);
  }

  // ---- rgb head (NET:68-70), FP32 on the VALU --------------------------------
  float part[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c)
        part[c] = __builtin_fmaf(acc8[m][r], hd[head_lds(kHeadRgbW) + c * 128 + g4 * 32 + 4 * m + r], part[c]);
  float rgb[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) rgb[c] = quad_sum(part[c]) + hd[head_lds(kHeadRgbB) + c];
  if (valid && g4 == 0) raw[gc] = make_float4(rgb[0], rgb[1], rgb[2], alpha);
  if constexpr (TRACE) {
    if (tr) trp[2] = __builtin_amdgcn_s_memtime();
  }
  R.rot = (R.rot + kNs) & 3;   // the next tile's slice 0 = this stream's slice kNs
  }
  // the last tile's wrapped DMA pieces land before the workgroup's LDS is freed
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (TRAIN) {   // one global max per output and workgroup
    __syncthreads();
    // (wave, lane), not threadIdx: the thread id is not kept live through the loop
    float* am = to.amax;
    asm volatile("" : "+s"(am));
    if (__builtin_amdgcn_readfirstlane(wave) == 0 && lane < 12)
      atomicMax(reinterpret_cast<unsigned*>(am) + lane, amax_lds[lane]);
  }
}

template <bool LIST>
__global__ __launch_bounds__(kX3Threads, 2) void mlp_x3_kernel(
    const float4* __restrict__ slices, const float* __restrict__ head,
    const float* __restrict__ rays_o, const float* __restrict__ rays_d,
    const float* __restrict__ z, int64_t z_stride, int64_t total, int S,
    float4* __restrict__ raw, const int* __restrict__ list, const int* __restrict__ count) {
  mlp_x3_body<LIST, false>(slices, head, rays_o, rays_d, z, z_stride, total, S, raw, list, count,
                           X3TrainOut{});
}

// Diagnostic twin of mlp_x3_kernel<false> (nerf_mlp_forward_x3_clock): the same
// body between two stamps of (s_memtime, s_memrealtime) per workgroup, written
// by its first lane to clk[4 b ..]: the shader clock the chip held during the
// launch is d memtime / d memrealtime x 100 MHz (MI355X_MICROARCH.md, DVFS
// give-back item 6). The production kernel carries no stamp.
__global__ __launch_bounds__(kX3Threads, 2) void mlp_x3_clock_kernel(
    const float4* __restrict__ slices, const float* __restrict__ head,
    const float* __restrict__ rays_o, const float* __restrict__ rays_d,
    const float* __restrict__ z, int64_t z_stride, int64_t total, int S,
    float4* __restrict__ raw, unsigned long long* __restrict__ clk,
    unsigned long long* __restrict__ trace) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  mlp_x3_body<false, false, true>(slices, head, rays_o, rays_d, z, z_stride, total, S, raw,
                                  nullptr, nullptr, X3TrainOut{}, trace);
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    ulonglong4 v;
    v.x = t0; v.y = t1; v.z = r0; v.w = r1;
    reinterpret_cast<ulonglong4*>(clk)[blockIdx.x] = v;
  }
}

// The training forward: sample p = ray * S + step at o + d * z (VR:165) as the
// inference kernel (nerf_mlp_train_forward_x3 passes rays_o = pts, rays_d =
// dirs, one shared zero depth and S = 1: o + d * 0 = o).
template <bool T16>
__global__ __launch_bounds__(kX3Threads, 2) void mlp_x3_train_kernel(
    const float4* __restrict__ slices, const float* __restrict__ head,
    const float* __restrict__ rays_o, const float* __restrict__ rays_d,
    const float* __restrict__ z, int64_t z_stride, int64_t total, int S,
    float4* __restrict__ raw, const X3TrainOut to) {
  mlp_x3_body<false, true, false, T16>(slices, head, rays_o, rays_d, z, z_stride, total, S, raw, nullptr,
                           nullptr, to);
}


// ===========================================================================
// The training backward through the MLP (the dgrad chain) in ONE launch: the
// inference kernel's per-tile body run through the transposed weights, from
// the loss gradient d raw [P][4] down to the encoding. Per 128-sample tile:
//   d_hv = (W_rgb^T d_rgb) * (hv > 0)                 (VALU, FP32; 128 rows)
//   D7   = (Wc^T d_hv + W_alpha^T d_sigma) * (h7 > 0)  (4 slices)
//   D_{i-1} = (W_i^T D_i) * (h_{i-1} > 0), i = 7 .. 1 (8 slices each; at i = 5
//   the h4 rows of W_5, with ENC first d_enc5 = W_5[:, :63]^T D5, 2 slices)
//   ENC: d_enc0 = W_0^T D0                            (2 slices)
// where Wc = W_views[:, :256] W_feat, the training step's fold of the feature
// layer (nerf_fold_views; feature = W_feat h7 + b_feat has no activation, so
// d h7 = W_feat^T W_views,feat^T d_hv + ...: one 128 -> 256 product instead of
// 128 -> 256 -> 256, and d feature never exists). (network.py:49-74's
// autograd; the layer launches of the unfused backward compute the same
// products unfolded.) Every output is written feature-major (the weight
// gradients read them) and its max |.| raised (their FP16 scales). The ReLU
// masks are the forward's bits, loaded one slice before the epilogue that
// applies them. Stream (pack: nerfhip.train_mlp.X3BwdStreamPacker): Wc^T (4),
// W_7^T, W_6^T (8 each), [W_5,enc^T (2)], W_5,h^T, W_4^T .. W_1^T (8 each),
// W_0^T (2): 64 slices (without ENC the 4 encoding slices are skipped).
// ===========================================================================
constexpr int kBwdScales = 3100;   // per-matrix weight scale exponents [11] in the head

struct X3BwdIO {
  const float4* d_raw;            // [P]: d rgb logits (x, y, z), d sigma (w)
  const unsigned short* bits[9];  // ReLU bits of h0..h7 (m_tiles 16), of the views output (8)
  float* d[12];                   // 0..7: D0..D7, 8: unused (DF: folded), 9: d_hv, 10: d_enc
                                  // (layer 5), 11: (layer 0)
  float* dmax;                    // raised: [i] = max |D_i|, [10] max |d_hv| ([8] untouched)
  float* d_raw_t;                 // nullable: rows 0..3 = d sigma, d rgb (x, y, z)
  Lay lay;                        // every output's layout (row stride / T16 block stride)
};

// Epilogue of a dgrad layer, fused into its last slice: 2^-shift * acc (exact),
// (+ rank-1 alpha-head term W_alpha[m] * d_sigma, layer 7), * mask bit; running
// |max|; into X[G] (FP32) for the next layer.
template <bool RANK1, bool MASK>
struct BwdEpi {
  Op (&X)[8];
  float inv;
  unsigned aw;          // LDS byte address of the lane group's packed alpha weights (RANK1)
  float dsig;
  float amax;
  unsigned mlds;        // LDS byte address of this lane's mask word of block 0 (MASK)
  unsigned mw[4];       // the mask words of the 4 tile blocks, read from LDS in the slice
  f32x4 bb[2][2];
  template <int G>
  __device__ __forceinline__ void prefetch() {
    if constexpr (MASK && (G & 1) == 0 && G < 8)   // drained with the next group's fragments
      asm volatile("ds_read_u16 %0, %1 offset:%2" : "=v"(mw[G >> 1]) : "v"(mlds), "i"(64 * G)
                   : "memory");
    if constexpr (RANK1 && G < 8) {
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bb[G & 1][0]) : "v"(aw), "i"(32 * G) : "memory");
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bb[G & 1][1]) : "v"(aw), "i"(32 * G + 16) : "memory");
    }
  }
  template <int G, typename Acc>
  __device__ __forceinline__ void after(Acc& acc) {
    if constexpr (G >= 1 && G <= 8) pair<G - 1>(acc);
  }
  template <typename Acc>
  __device__ __forceinline__ void finish(Acc& acc) {
    lds_drain();
    pair<7>(acc);
  }
  template <int G, typename Acc>
  __device__ __forceinline__ void pair(Acc& acc) {
    Op v;
    unsigned m = 0xffu;
    if constexpr (MASK) m = mw[G >> 1] >> (8 * (G & 1));
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a = acc[2 * G][r] * inv, b = acc[2 * G + 1][r] * inv;   // exact: power of two
      if constexpr (RANK1) {
        a = __builtin_fmaf(bb[G & 1][0][r], dsig, a);
        b = __builtin_fmaf(bb[G & 1][1][r], dsig, b);
      }
      v[r] = ((m >> r) & 1u) ? a : 0.0f;
      v[4 + r] = ((m >> (4 + r)) & 1u) ? b : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < 8; j += 2)
      asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(amax) : "v"(v[j]), "v"(v[j + 1]));
    asm volatile("" : "+v"(v), "+v"(amax));
    X[G] = v;
  }
};

// The mask words of one layer's ReLU bits for this (tile, wave): 4 x 64 u16
// (x3_layer_kernel's MT 16 layout, 512 B contiguous) staged into the wave's
// LDS area by two LDS-DMA dwords per lane, a slice before the epilogue that
// reads them (an ordinary load's result would make hipcc wait with a vmcnt
// that ignores LDS-DMA, i.e. drain the weight stream). The loader waves' slice
// end certifies them (they are older than that slice's pieces); the other
// waves wait vmcnt(0) at the end of the slice (wait_nonloader).
struct MaskSrc {
  __amdgpu_buffer_rsrc_t rs;
  unsigned soff;        // uniform: ((tile * 8 + wave) * 4 * 64) * 2
  float* dst;           // this wave's 512-B LDS area
  __device__ __forceinline__ void load() const {
    unsigned lid = __lane_id();
    asm volatile("" : "+v"(lid));
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)dst, 4, (int)(lid * 4u), (int)soff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(dst + 64), 4, (int)(lid * 4u),
                                             (int)(soff + 256), 0, 0);
  }
};

// slice hook: the previous output's pair P stored, the epilogue's masks loaded
// (both before the slice's DMA pieces), then an operand split
template <int P, typename Pend, typename Split>
struct StoreMaskThen {
  Pend& st;
  Split sp;
  const MaskSrc& ms;
  bool loader;          // wave-uniform: this wave stages weight pieces (waves 0-3)
  template <int G>
  __device__ __forceinline__ void prefetch() {
    if constexpr (G == 0) ms.load();
  }
  template <int G, typename Acc>
  __device__ __forceinline__ void after(Acc& acc) {
    if constexpr (P >= 0) store_pair_at<P, G>(st, sp.op);   // behind group 0's MFMAs
    sp.template after<G>(acc);
    if constexpr (G == 7) {
      if (!loader) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
};
struct NoSplit {   // operands already split (the D4 pass after the encoding rows)
  template <int G, typename Acc>
  __device__ __forceinline__ void after(Acc&) {}
};

// The 8 slices of a 256-row dgrad layer over operand array X: slice q stores the
// previous output's pair q+1 and splits operand q+1 (unless PRESPLIT), slice 6
// also loads the masks, slice 7 runs the epilogue.
template <bool PRESPLIT, typename Epi, typename Pend>
__device__ __forceinline__ void dgrad_slices(f32x4 (&acc)[16], const Ring& R, int g, Op (&X)[8],
                                             float s, FragPipe& fp, Epi& epi, Pend& st,
                                             const MaskSrc& ms) {
  if constexpr (PRESPLIT) {
    NoHook nh;
    slice256x<0, true>(acc, R, g + 0, X, fp, nh);
    slice256<1>(acc, R, g + 1, X, fp, nh);
    slice256<2>(acc, R, g + 2, X, fp, nh);
    slice256<3>(acc, R, g + 3, X, fp, nh);
    slice256<4>(acc, R, g + 4, X, fp, nh);
    slice256<5>(acc, R, g + 5, X, fp, nh);
    { StoreMaskThen<-1, Pend, NoSplit> h{st, {}, ms, R.wave < 4};
      slice256<6>(acc, R, g + 6, X, fp, h); }
  } else {
    { StoreThen<1, Pend, SplitHook> h{st, {X[1], s}}; slice256x<0, true>(acc, R, g + 0, X, fp, h); }
    { StoreThen<2, Pend, SplitHook> h{st, {X[2], s}}; slice256<1>(acc, R, g + 1, X, fp, h); }
    { StoreThen<3, Pend, SplitHook> h{st, {X[3], s}}; slice256<2>(acc, R, g + 2, X, fp, h); }
    { StoreThen<4, Pend, SplitHook> h{st, {X[4], s}}; slice256<3>(acc, R, g + 3, X, fp, h); }
    { StoreThen<5, Pend, SplitHook> h{st, {X[5], s}}; slice256<4>(acc, R, g + 4, X, fp, h); }
    { StoreThen<6, Pend, SplitHook> h{st, {X[6], s}}; slice256<5>(acc, R, g + 5, X, fp, h); }
    { StoreMaskThen<7, Pend, SplitHook> h{st, {X[7], s}, ms, R.wave < 4};
      slice256<6>(acc, R, g + 6, X, fp, h); }
  }
  slice256<7>(acc, R, g + 7, X, fp, epi);
  epi.finish(acc);
}

template <bool ENC, bool T16>
__global__ __launch_bounds__(kX3Threads, 2) void mlp_x3_bwd_kernel(
    const float4* __restrict__ slices, const float* __restrict__ head, int64_t P,
    const X3BwdIO io) {
  __shared__ __attribute__((aligned(16))) float ring[4 * kSliceFloats];
  __shared__ __attribute__((aligned(16))) float hd[kHeadLds];
  __shared__ unsigned dmax_lds[13];
  __shared__ __attribute__((aligned(16))) float mask_lds[8 * 128];   // 512 B per wave
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  Ring R{ring, slices, wave, lane};
  constexpr int kNs = ENC ? 64 : 60;
  for (int t = 0; t < kX3DmaAhead; ++t)   // all 8 waves, 4 pieces each
    stage_slice(make_dma_blocks(slices, t, R.buf(t), wave * kBlocksPerWave, wave, lane, true, 64));
  load_head_lds(hd, head, tid, kX3Threads);
  if (tid < 13) dmax_lds[tid] = 0u;

  FragPipe fp;
  fp.ns = kNs;
  fp.nphys = 64;
  if (!ENC) fp.gap = 20;   // the encoding slices 20, 21 skipped (62, 63: past the end)
  const int64_t ntiles = (P + kX3Tile - 1) / kX3Tile;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
  const bool first_tile = tile == (int64_t)blockIdx.x;
  const int64_t gs = tile * kX3Tile + wave * 16 + (lane & 15);
  int g4 = lane >> 4;
  asm volatile("" : "+v"(g4));
  const bool valid = gs < P;
  const int64_t gl = valid ? gs : P - 1;
  // samples past P: d raw 0, so every product of theirs is 0 whatever the
  // (unwritten) mask words of their tile say, and no max |.| sees them
  float4 dr = io.d_raw[gl];
  if (!valid) dr = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (io.d_raw_t && g4 == 0 && valid) {   // d raw as rows: the heads' wgrad operands
    // d sigma at row 0, d rgb at rows 1..3 (feature-major) or 16..18 (T16: the
    // rgb head's operand starts a 16-row group of its own, BlockRows). Rows
    // 1..15 of T16 stay unwritten: the shared views-encoding / rgb wgrad tile
    // reads them as A rows 129..143, whose products land in output rows of
    // their own (an MFMA row only meets its own A row; the split scale comes
    // from the tensor maxima, not from the data) and are discarded. (Zeroing
    // them here -- five more stores per lane group ahead of the slices'
    // counted vmcnt waits -- was followed by an intermittent illegal address:
    // reverted)
    constexpr int kRgb = T16 ? 16 : 1;
    char* t = reinterpret_cast<char*>(io.d_raw_t);
    *reinterpret_cast<float*>(t + io.lay.template elem<T16>(0, gs)) = dr.w;
    *reinterpret_cast<float*>(t + io.lay.template elem<T16>(kRgb, gs)) = dr.x;
    *reinterpret_cast<float*>(t + io.lay.template elem<T16>(kRgb + 1, gs)) = dr.y;
    *reinterpret_cast<float*>(t + io.lay.template elem<T16>(kRgb + 2, gs)) = dr.z;
  }
  // outputs / masks of this (tile, wave): pointers loaded at their layer
  auto store_for = [&](int k, int rows) {
    ActStore st;
    int ki = k;
    asm volatile("" : "+s"(ki));
    st.rs = rows_rsrc<T16>(io.d[ki], rows, io.lay);
    st.on = io.d[ki] != nullptr;
    st.rb = __builtin_amdgcn_make_buffer_rsrc((void*)io.d[ki], 0, 0, 0x00020000);
    st.template set_lay<T16>(io.lay, tile, wave);
    st.sboff = 0u;
    st.wb = 0u;
    st.bits = false;
    st.valid = valid;
    return st;
  };
  // the bit words of whole 128-sample tiles (relu_bits_words): 4 KiB per tile
  const int mask_bytes = (int)(ntiles * 8 * 4 * 64 * 2);
  auto mask_for = [&](int L) {
    int li = L;
    asm volatile("" : "+s"(li));
    return MaskSrc{__builtin_amdgcn_make_buffer_rsrc((void*)io.bits[li], 0, mask_bytes, 0x00020000),
                   (unsigned)(((tile * 8 + wave) * 4 * 64) * 2), mask_lds + wave * 128};
  };
  auto amax_to_lds = [&](int slot, float mx) { lds_max_u32(&dmax_lds[slot], __float_as_uint(mx)); };

  const unsigned mlane = lds_addr(mask_lds + wave * 128) + lane * 2u;   // block k: + 128 k
  f32x4 acc[16];
  Op X[8];
  if (first_tile) __syncthreads();   // head, d raw and the three prologue slices resident
  // max |d rgb| and |d sigma| (the heads' wgrad scales, slots 11 / 12): every
  // lane group holds its samples' d raw, so lane group 0 reports. After the
  // first tile's barrier: wave 0's zeroing of the slots (above) must land first
  if (g4 == 0) {
    lds_max_u32(&dmax_lds[11], __float_as_uint(fmaxf(fmaxf(fabsf(dr.x), fabsf(dr.y)), fabsf(dr.z))));
    lds_max_u32(&dmax_lds[12], __float_as_uint(fabsf(dr.w)));
  }
  load_frags<0>(fp.x, lds_base(R.buf(0), lane));

  float mx;   // max |.| of the last product (its FP16 split scale)
  // ---- d_hv = (W_rgb^T d_rgb) * (hv > 0), NET:68-70 backward, FP32 on the VALU
  {
    int i8 = 8;
    asm volatile("" : "+s"(i8));
    const unsigned short* bv = io.bits[i8];
    const int64_t wv0 = ((tile * 8 + wave) * 2) * 64 + lane;     // views bits: MT 8
    const unsigned mv0 = bv[wv0], mv1 = bv[wv0 + 64];
    const float* wr = hd + head_lds(kHeadRgbW) + g4 * 32;
    mx = 0.0f;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = 2 * q + (j >> 2), r = j & 3;
        float v = wr[4 * m + r] * dr.x;                        // sum over c in order
        v = __builtin_fmaf(wr[128 + 4 * m + r], dr.y, v);
        v = __builtin_fmaf(wr[256 + 4 * m + r], dr.z, v);
        const unsigned mw = m < 4 ? mv0 : mv1;
        v = ((mw >> (4 * (m & 3) + r)) & 1u) ? v : 0.0f;
        X[4 + q][j] = v;   // operands 4..7: the last slice reads only X[7]
        mx = fmaxf(mx, fabsf(v));
      }
    ActStore sv = store_for(9, 128);
    sv.template pair<0>(X[4]);
    sv.template pair<1>(X[5]);
    sv.template pair<2>(X[6]);
    sv.template pair<3>(X[7]);
    amax_to_lds(10, mx);
    const int e = act_exponent(sample_max(mx));
    const float s = ldexpf(1.0f, e);
    split_op(X[4], s);
    // ---- D7 = (Wc^T d_hv + W_alpha^T d_sigma) * (h7 > 0) (NET:61, 63-65):
    // 4 slices over operands 4..7, so the epilogue's writes of X[0..6] in the
    // last slice miss its operand; the view encoding rows are not needed (view
    // directions are constants). h7's mask words load in slice 2.
    BwdEpi<true, true> epi{X, ldexpf(1.0f, -((int)hd[head_lds(kBwdScales) + 0] + e)),
                           lds_addr(hd + kLdsAlphaW + g4 * kLdsGroup), dr.w, 0.0f, mlane};
    const MaskSrc ms = mask_for(7);
    { SplitHook h{X[5], s}; slice256x<4, true>(acc, R, 0, X, fp, h); }
    { SplitHook h{X[6], s}; slice256<5>(acc, R, 1, X, fp, h); }
    { StoreMaskThen<-1, ActStore, SplitHook> h{sv, {X[7], s}, ms, R.wave < 4};
      slice256<6>(acc, R, 2, X, fp, h); }
    slice256<7>(acc, R, 3, X, fp, epi);
    epi.finish(acc);
    amax_to_lds(7, epi.amax);
    mx = epi.amax;
  }
  int g = 4;
  ActStore st;
  int e;
  float s;
  // ---- D_{i-1} = (W_i^T D_i) * (h_{i-1} > 0), i = 7 .. 1 ---------------------
  for (int i = 7; i >= 1; --i) {
    st = store_for(i, 256);           // D_i rows
    st.template pair<0>(X[0]);
    e = act_exponent(sample_max(mx));
    s = ldexpf(1.0f, e);
    const int sidx = i >= 6 ? 9 - i : (i == 5 ? 5 : 10 - i);   // W7 2, W6 3, W5h 5, W4 6 .. W1 9
    BwdEpi<false, true> epi{X, ldexpf(1.0f, -((int)hd[head_lds(kBwdScales) + sidx] + e)), 0u, 0.0f, 0.0f,
                            mlane};
    const MaskSrc ms = mask_for(i - 1);
    if (ENC && i == 5) {
      // the encoding rows first (they read D5 too): D5 stored and split whole
      st.template pair<1>(X[1]); st.template pair<2>(X[2]); st.template pair<3>(X[3]);
      st.template pair<4>(X[4]); st.template pair<5>(X[5]); st.template pair<6>(X[6]);
      st.template pair<7>(X[7]);
#pragma unroll
      for (int q = 0; q < 8; ++q) split_op(X[q], s);
      NoHook nh;
      run_slice3<8, StepEnc4<0, true>>(acc, R, g, X, fp, nh); x3_slice_end<2>(fp);
      run_slice3<8, StepEnc4<4>>(acc, R, g + 1, X, fp, nh); x3_slice_end<2>(fp);
      g += 2;
      {   // d_enc5 = 2^-shift acc (rows 0..63), straight to HBM
        ActStore se = store_for(10, 64);
        const float inv = ldexpf(1.0f, -((int)hd[head_lds(kBwdScales) + 4] + e));
        Op v0, v1;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v0[r] = acc[0][r] * inv; v0[4 + r] = acc[1][r] * inv;
          v1[r] = acc[2][r] * inv; v1[4 + r] = acc[3][r] * inv;
        }
        se.template pair<0>(v0);
        se.template pair<1>(v1);
      }
      dgrad_slices<true>(acc, R, g, X, s, fp, epi, st, ms);
    } else {
      split_op(X[0], s);
      dgrad_slices<false>(acc, R, g, X, s, fp, epi, st, ms);
    }
    g += 8;
    amax_to_lds(i - 1, epi.amax);
    mx = epi.amax;
  }
  // X holds D0 (FP32)
  st = store_for(0, 256);
  st.template pair<0>(X[0]); st.template pair<1>(X[1]); st.template pair<2>(X[2]);
  st.template pair<3>(X[3]); st.template pair<4>(X[4]); st.template pair<5>(X[5]);
  st.template pair<6>(X[6]); st.template pair<7>(X[7]);
  if constexpr (ENC) {   // ---- d_enc0 = W_0^T D0 (64 rows)
    e = act_exponent(sample_max(mx));
    s = ldexpf(1.0f, e);
#pragma unroll
    for (int q = 0; q < 8; ++q) split_op(X[q], s);
    NoHook nh;
    run_slice3<8, StepEnc4<0, true>>(acc, R, g, X, fp, nh); x3_slice_end<2>(fp);
    run_slice3<8, StepEnc4<4>>(acc, R, g + 1, X, fp, nh); x3_slice_end<2>(fp);
    ActStore se = store_for(11, 64);
    const float inv = ldexpf(1.0f, -((int)hd[head_lds(kBwdScales) + 10] + e));
    Op v0, v1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v0[r] = acc[0][r] * inv; v0[4 + r] = acc[1][r] * inv;
      v1[r] = acc[2][r] * inv; v1[4 + r] = acc[3][r] * inv;
    }
    se.template pair<0>(v0);
    se.template pair<1>(v1);
  }
  R.rot = (R.rot + kNs) & 3;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float* dm = io.dmax;
  asm volatile("" : "+s"(dm));
  if (wave == 0 && lane < 13 && lane != 9)
    atomicMax(reinterpret_cast<unsigned*>(dm) + lane, dmax_lds[lane]);
}


// ===========================================================================
// Training (BASELINE configs[2]): the MLP of a training
// step as x3 MFMA GEMMs over feature-major activations in HBM ([F][P]: row f
// holds feature f of every sample p). nerfhip/train_mlp.py chains them:
//   forward  h_L = act(W_L h_{L-1} + b_L)          x3_layer_kernel (bias, ReLU)
//   dgrad    d_{L-1} = (W_L^T d_L) * (h_{L-1} > 0)  x3_layer_kernel (W^T, mask)
//   wgrad    dW_L = d_L h_{L-1}^T (sum over P)      x3_wgrad_kernel (split-K)
// (network.py:49-74 and its autograd; no reference kernel computes these.)
// Same 3-term FP16 split as the inference kernel: per-sample activation
// scales in the layer kernel (K = features), per-tensor scales in wgrad
// (K = samples: one scale along K).
// ===========================================================================
constexpr int kTrainThreads = 512;   // 8 waves x 16 samples
constexpr int kTrainTile = 128;

__device__ __forceinline__ void vm_wait_slices(int n_pieces) {
  // wait until at most n_pieces of this wave's LDS-DMA pieces are in flight
  if (n_pieces >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n_pieces >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n_pieces >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (n_pieces >= 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The K step's groups; with nxt, the next K step's operand is split (FP32 ->
// FP16 hi/lo at scale s, as split_op) in the MFMA shadows of the even groups,
// 8 / NG value pairs each, into t, committed to *nxt after the last group (it
// is not read by this K step). Same values as splitting it up front.
template <int G, int NG>
__device__ __forceinline__ void layer_groups(f32x4* acc, unsigned base, const Op& b, Frags& x,
                                             Frags& y, Op* nxt = nullptr, float s = 0.0f,
                                             Op* t = nullptr) {
  if constexpr (G < NG) {
    lds_drain();
    if constexpr (G + 1 < NG) {
      if constexpr ((G & 1) == 0) load_frags<G + 1>(y, base);
      else load_frags<G + 1>(x, base);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((G & 1) == 0) mfma3x2<false>(acc[2 * G], acc[2 * G + 1], x, b);
    else mfma3x2<false>(acc[2 * G], acc[2 * G + 1], y, b);
    if constexpr ((G & 1) == 0) {
      constexpr int kPairs = 8 / NG;   // value pairs split after this group
      if (nxt) {
#pragma unroll
        for (int i = 0; i < kPairs; ++i) {
          constexpr int k0 = (G / 2) * kPairs;
          float hp, lp;
          split2((*nxt)[2 * (k0 + i)], (*nxt)[2 * (k0 + i) + 1], s, hp, lp);
          asm volatile("" : "+v"(hp), "+v"(lp));
          (*t)[k0 + i] = hp;
          (*t)[4 + k0 + i] = lp;
        }
      }
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);   // up to 2 VALU
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (G + 1 == NG) {
      if (nxt) *nxt = *t;
    }
    layer_groups<G + 1, NG>(acc, base, b, x, y, nxt, s, t);
  }
}

// C[m][p] = epi(2^-(sw+e_p) * sum_k W[m][k] * B[k][p]), m < 16*MT, k < 32*NK:
//   + bias[m] (optional), + ru[m] * rw[p] (optional rank-1 term), ReLU
//   (optional), * (mask[m][p] > 0) (optional). W packed by pack_x3_matrix
//   (nerfhip/train_mlp.py): slice q = K step q, block 2t + part = tile t hi/lo,
//   lane l -> row 16t + (l & 15), k = 32q + 8(l >> 4) + j.
// Persistent: a workgroup walks sample tiles of 128 (tile, tile + gridDim.x,
// ...); W streams L2 -> LDS through a 4-deep ring of slices that runs on
// across tiles, and after slice q of a tile the registers of its B operand are
// refilled with K step q of the NEXT tile, so those HBM loads land while the
// rest of the tile computes. Each tile ends with vmcnt(0): within a tile the
// counted wait before a slice barrier then only counts that tile's operations.
// epilogue terms, a compile-time set (no per-element branches or waits)
// kEpiMaskBits: the mask as one bit per element (written by a forward launch
// with kEpiOutBits: bit (C > 0) of its ReLU output) instead of an FP32 tensor,
// in this kernel's own lane layout (so the consumer has the producer's MT):
// per block of 4 tiles a lane keeps the 16 bits of its sample (tile * 128 +
// wave * 16 + (lane & 15)) and rows 16 (u0 + t) + 4 (lane >> 4) + r, bit
// 4 t + r, as one u16 at ((tile * 8 + wave) * MT / 4 + u0 / 4) * 64 + lane:
// 32 B per sample and 256-row layer instead of the 1 KiB of the FP32 mask.
// kEpiHead: a head of n_head (1..3) outputs on the final C of the sample,
// head_out[p * 4 + head_col + c] = sum_m head_w[c][m] C[m][p] + head_b[c] (the
// alpha head on h7 and the rgb head on the views output, NET:61, 68-70,
// written straight into raw [P][4]): no second pass over C.
enum : int { kEpiBias = 1, kEpiRelu = 2, kEpiMask = 4, kEpiRank1 = 8, kEpiMaskBits = 16,
             kEpiOutBits = 32, kEpiHead = 64 };

__device__ __forceinline__ void vm_wait_n(int n) {   // s_waitcnt vmcnt(n), n uniform
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 25: asm volatile("s_waitcnt vmcnt(25)" ::: "memory"); break;
    case 26: asm volatile("s_waitcnt vmcnt(26)" ::: "memory"); break;
    case 28: asm volatile("s_waitcnt vmcnt(28)" ::: "memory"); break;
    case 32: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

template <int MT, int NK, int EPI>
__global__ __launch_bounds__(kTrainThreads, 2) void x3_layer_kernel(
    const uint4* __restrict__ slices, const int* __restrict__ sw_ptr,
    const float* __restrict__ bias, const float* __restrict__ B, int64_t ldb,
    const float* __restrict__ mask, int64_t ldm, const float* __restrict__ ru,
    const float* __restrict__ rw, float* __restrict__ C, int64_t ldc, int64_t P,
    float* __restrict__ amax_out, unsigned short* __restrict__ bits_out,
    const unsigned short* __restrict__ bits_in, const float* __restrict__ head_w,
    const float* __restrict__ head_b, int n_head, float* __restrict__ head_out, int head_col) {
  constexpr int kPieces = 2 * MT;          // 1-KiB LDS-DMA pieces per slice
  constexpr int kSliceU4 = kPieces * 64;
  constexpr int kPpw = kPieces / 8;        // pieces per wave
  static_assert(kPieces % 8 == 0, "MT must be a multiple of 4");
  __shared__ __attribute__((aligned(16))) uint4 ring[4 * kSliceU4];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g4 = lane >> 4;
  const int64_t ntiles = (P + kTrainTile - 1) / kTrainTile;
  const int64_t t0 = blockIdx.x, tstride = gridDim.x;
  const int nt = t0 < ntiles ? (int)((ntiles - 1 - t0) / tstride + 1) : 0;   // this WG's tiles
  const int total = nt * NK;                                                  // its slices

  // slice g of this workgroup's stream = K step g % NK, in ring slot g & 3;
  // buffer-form LDS-DMA: the lane offset is constant, the slice offset an SGPR
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc(
      (void*)slices, 0, NK * kSliceU4 * 16, 0x00020000);
  auto stage = [&](int g) {
    if (g < total) {
      const int q = g % NK;
#pragma unroll
      for (int i = 0; i < kPpw; ++i) {
        const int b = wave + 8 * i;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rW, (lds_ptr_t)(ring + (g & 3) * kSliceU4 + b * 64), 16, (b * 64 + lane) * 16,
            __builtin_amdgcn_readfirstlane(q * kSliceU4 * 16), 0, 0);
      }
    }
  };
  stage(0);
  stage(1);
  stage(2);

  auto sample_of = [&](int64_t tile) {
    return tile * kTrainTile + wave * 16 + (lane & 15);
  };
  // HBM operands as buffer resources: a lane's offset is one 32-bit VGPR, the
  // row offset an SGPR, and a sample past P reads 0 / drops its store (offset
  // pushed past num_records) -- no per-load address registers or branches
  const int nbB = (int)(32 * NK * ldb * 4);
  const int nbC = (int)(16 * MT * ldc * 4);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)B, 0, nbB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rC = __builtin_amdgcn_make_buffer_rsrc((void*)C, 0, nbC, 0x00020000);
  const int nbM = mask ? (int)(16 * MT * ldm * 4) : 0;
  const __amdgpu_buffer_rsrc_t rM =
      __builtin_amdgcn_make_buffer_rsrc((void*)(mask ? mask : B), 0, nbM, 0x00020000);
  // row 32 q + 8 g4 + j of sample p: VGPR offset (8 g4 + j) rows + p (8 per
  // lane, one per j), SGPR offset 32 q rows (one per K step)
  const unsigned ldb4 = (unsigned)ldb * 4u;
  struct VOff { unsigned o[8]; };
  auto voff_b = [&](int64_t p) {
    VOff v;
    const unsigned base = p < P ? (unsigned)(((int64_t)8 * g4 * ldb + p) * 4) : (unsigned)nbB;
#pragma unroll
    for (int j = 0; j < 8; ++j) v.o[j] = base + (unsigned)j * ldb4;
    return v;
  };
  auto load_b = [&](int q, const VOff& vo, Op& dst) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      dst[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                             rB, (int)vo.o[j], (int)(32u * q * ldb4), 0));
  };
  Op b[NK];
  {
    const VOff vo = voff_b(sample_of(t0));
#pragma unroll
    for (int q = 0; q < NK; ++q) load_b(q, vo, b[q]);
  }
  __syncthreads();   // prologue slices landed (hipcc waits vmcnt(0) before the barrier)

  const int sw = *sw_ptr;
  float omax = 0.0f;   // max |C| of this lane's stored values (for amax_out)
  int g = 0;
  for (int it = 0; it < nt; ++it) {
    const int64_t tile = t0 + (int64_t)it * tstride;
    const int64_t p = sample_of(tile);
    const bool valid = p < P;
    const int64_t pc = valid ? p : P - 1;
    const bool has_next = it + 1 < nt;
    const VOff von = voff_b(sample_of(tile + tstride));
    float mx = 0.0f;   // (samples past P loaded as 0)
#pragma unroll
    for (int q = 0; q < NK; ++q) mx = fmaxf(mx, op_absmax(b[q]));
    const int e = act_exponent(sample_max(mx));
    const float s = ldexpf(1.0f, e);
    split_op(b[0], s);   // b[1..NK-1] in the MFMA shadows of the K loop
    Op split_tmp;

    f32x4 acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = f32x4(0.0f);

#pragma unroll
    for (int q = 0; q < NK; ++q, ++g) {
      stage(g + 3);
      const unsigned base = lds_base((const float*)(ring + (g & 3) * kSliceU4), lane);
      Frags x, y;
      load_frags<0>(x, base);
      if (q + 1 < NK) layer_groups<0, MT / 2>(acc, base, b[q], x, y, &b[q + 1], s, &split_tmp);
      else layer_groups<0, MT / 2>(acc, base, b[q], x, y);
      if (has_next) load_b(q, von, b[q]);   // K step q of the next tile, registers just freed
      if (g + 1 < total) {   // slice g+1 landed (this wave's pieces), then visible to all
        if (q >= 2) {
          // younger than the pieces of g+1 (issued at slice q-2 of this tile): the
          // next-tile loads of slices q-2..q and the pieces of g+2, g+3
          vm_wait_n(24 * (int)has_next + kPpw * ((g + 2 < total) + (g + 3 < total)));
        }   // q < 2: those pieces were issued before this tile's closing vmcnt(0)
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
    }

    const float inv = ldexpf(1.0f, -(sw + e));
    // row 16 t + 4 g4 + r: VGPR offset (4 g4 + r) rows + p, SGPR offset 16 t rows
    const unsigned ldc4 = (unsigned)ldc * 4u, ldm4 = (unsigned)ldm * 4u;
    unsigned voc[4], vom[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      voc[r] = valid ? (unsigned)(((int64_t)(4 * g4 + r) * ldc + p) * 4) : (unsigned)nbC;
      vom[r] = valid ? (unsigned)(((int64_t)(4 * g4 + r) * ldm + p) * 4) : (unsigned)nbM;
    }
    float hpart[3] = {0.0f, 0.0f, 0.0f};   // kEpiHead: this lane's share of each output
    // epilogue in blocks of 4 tiles: every load of a block issued before its use
#pragma unroll
    for (int u0 = 0; u0 < MT; u0 += 4) {
      float v[4][4], mk[4][4];
      // this block's 16 mask bits of this lane (u16 word)
      const int64_t wb = (((tile * 8 + wave) * MT + u0) / 4) * 64 + lane;
      unsigned mbits = 0u;
      if constexpr ((EPI & kEpiMaskBits) != 0) mbits = bits_in[wb];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 16 * (u0 + t) + 4 * g4 + r;
          v[t][r] = acc[u0 + t][r] * inv;   // exact: power of two
          if constexpr ((EPI & kEpiMask) != 0)
            mk[t][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                     rM, (int)vom[r], (int)(16u * (u0 + t) * ldm4), 0));
          if constexpr ((EPI & kEpiBias) != 0) v[t][r] = v[t][r] + bias[m];
          if constexpr ((EPI & kEpiRank1) != 0) v[t][r] = __builtin_fmaf(ru[m], rw[pc], v[t][r]);
        }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if constexpr ((EPI & kEpiRelu) != 0) v[t][r] = fmaxf(v[t][r], 0.0f);
          if constexpr ((EPI & kEpiMask) != 0) v[t][r] = mk[t][r] > 0.0f ? v[t][r] : 0.0f;
          if constexpr ((EPI & kEpiMaskBits) != 0)
            v[t][r] = ((mbits >> (4 * t + r)) & 1u) ? v[t][r] : 0.0f;
        }
      if constexpr ((EPI & kEpiOutBits) != 0) {
        // bit 4 t + r = (v > 0): post-ReLU v >= 0, so min(bits(v), 1)
        unsigned mine = 0u;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            mine |= min(__float_as_uint(v[t][r]), 1u) << (4 * t + r);
        if (valid) bits_out[wb] = (unsigned short)mine;
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {   // a sample past P: offset past num_records, dropped
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[t][r]), rC,
                                                (int)voc[r], (int)(16u * (u0 + t) * ldc4), 0);
          omax = valid ? fmaxf(omax, fabsf(v[t][r])) : omax;
        }
      if constexpr ((EPI & kEpiHead) != 0) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          if (c < n_head) {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              const float4 hw = *reinterpret_cast<const float4*>(
                  head_w + c * 16 * MT + 16 * (u0 + t) + 4 * g4);
              hpart[c] = __builtin_fmaf(v[t][0], hw.x, hpart[c]);
              hpart[c] = __builtin_fmaf(v[t][1], hw.y, hpart[c]);
              hpart[c] = __builtin_fmaf(v[t][2], hw.z, hpart[c]);
              hpart[c] = __builtin_fmaf(v[t][3], hw.w, hpart[c]);
            }
          }
        }
      }
    }
    if constexpr ((EPI & kEpiHead) != 0) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        if (c < n_head) {
          const float h = quad_sum(hpart[c]) + head_b[c];
          if (valid && g4 == 0) head_out[p * 4 + head_col + c] = h;
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the next tile starts clean
  }
  if (amax_out) {   // one atomic per workgroup (as ordered uint bits: values >= 0)
    __shared__ unsigned wg_max;
    if (threadIdx.x == 0) wg_max = 0u;
    __syncthreads();
    atomicMax(&wg_max, __float_as_uint(omax));   // LDS atomics
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(reinterpret_cast<unsigned*>(amax_out), wg_max);
  }
}

// Partial weight gradients: part[c][m][n] = sum over the samples of subset c
// (32-sample steps c, c + C, c + 2C, ... of C = ceil(P / chunk) subsets) of
// A[m][p] * B[n][p] (A = dL/d(pre-activation) [M][P], B = layer input [N][P],
// both feature-major); bias_part[c][m] = sum over the chunk of A[m][p].
// Per-tensor power-of-two scales from amax_a / amax_b (device scalars: max |A|,
// max |B|) keep the FP16 splits in range; undone exactly at the end.
// Workgroup tile 256 (m) x 256 (n): every A and B element of a chunk is read
// from HBM once. K steps of 32 samples are staged through LDS already split
// (hi, lo) in MFMA fragment layout, double-buffered, the next step's global
// loads in flight during the current step's MFMAs. Wave tile 64 x 128: its
// 4 A fragments stay in registers while the 8 B fragments stream past them.
constexpr int kWgTile = 256;
__global__ __launch_bounds__(kTrainThreads, 2) void x3_wgrad_kernel(
    const float* __restrict__ A, int64_t lda, int M, const float* __restrict__ B, int64_t ldb,
    int N, int64_t P, int64_t chunk, const float* __restrict__ amax_a,
    const float* __restrict__ amax_b, float* __restrict__ part, float* __restrict__ bias_part) {
  // [stage][A|B][16 tiles x (hi, lo)][64 lanes] x 16 B = 2 x 2 x 32 KiB
  __shared__ __attribute__((aligned(16))) uint4 lds[2][2][32 * 64];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int m0 = blockIdx.x * kWgTile, n0 = blockIdx.y * kWgTile;
  // K steps of 32 samples interleaved over the gridDim.z workgroups of an output
  // tile (step z, z + Z, ...): the concurrently running workgroups read
  // neighbouring samples of every row (DRAM page locality)
  const int64_t pb = (int64_t)blockIdx.z * 32;
  const int64_t pe = P;
  const int64_t kstride = (int64_t)gridDim.z * 32;
  (void)chunk;
  const int ea = act_exponent(*amax_a), eb = act_exponent(*amax_b);
  const float sa = ldexpf(1.0f, ea), sb = ldexpf(1.0f, eb);

  // staging units: u = tid + 512 i (i = 0, 1) -> row u >> 2, samples 8 (u & 3) + 0..7
  const float* ap[2];
  const float* bp[2];
  bool aok[2], bok[2];
  int slot[2], off[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int u = tid + 512 * i, row = u >> 2, gq = u & 3;
    aok[i] = m0 + row < M;
    bok[i] = n0 + row < N;
    ap[i] = A + (int64_t)(aok[i] ? m0 + row : 0) * lda;
    bp[i] = B + (int64_t)(bok[i] ? n0 + row : 0) * ldb;
    off[i] = 8 * gq;
    slot[i] = ((row >> 4) * 2) * 64 + (row & 15) + 16 * gq;   // hi block; lo = +64
  }
  auto load8 = [&](const float* src, bool ok, int64_t p0, float (&v)[8]) {
    // p0 = this unit's first sample (chunk start + 32 k + 8 gq)
    if (ok && p0 + 8 <= pe && ((((uintptr_t)(src + p0)) & 15) == 0)) {
      const float4 x = *reinterpret_cast<const float4*>(src + p0);
      const float4 y = *reinterpret_cast<const float4*>(src + p0 + 4);
      v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (ok && p0 + j < pe) ? src[p0 + j] : 0.0f;
    }
  };
  auto put = [&](const float (&v)[8], float sc, uint4* dst, int sl) {
    float hp[4], lp[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) split2(v[2 * k], v[2 * k + 1], sc, hp[k], lp[k]);
    dst[sl] = make_uint4(__float_as_uint(hp[0]), __float_as_uint(hp[1]), __float_as_uint(hp[2]),
                         __float_as_uint(hp[3]));
    dst[sl + 64] = make_uint4(__float_as_uint(lp[0]), __float_as_uint(lp[1]),
                              __float_as_uint(lp[2]), __float_as_uint(lp[3]));
  };

  const int mb = wave & 3, nb = wave >> 2;   // wave tile: rows 64 mb.., cols 128 nb..
  const bool busy = (m0 + 64 * mb < M) && (n0 + 128 * nb < N);   // wave-uniform
  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4(0.0f);

  float va[2][8], vb[2][8];
  float rsum[2] = {0.0f, 0.0f};   // shares of sum_p A[row][p] (bias gradient)
  int st = 0;
  if (pb < pe) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      load8(ap[i], aok[i], pb + off[i], va[i]);
      load8(bp[i], bok[i], pb + off[i], vb[i]);
    }
  }
  for (int64_t k0 = pb; k0 < pe; k0 += kstride) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) rsum[i] += va[i][j];
      put(va[i], sa, lds[st][0], slot[i]);
      put(vb[i], sb, lds[st][1], slot[i]);
    }
    __syncthreads();
    if (k0 + kstride < pe) {   // next K step's loads in flight during the MFMAs
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        load8(ap[i], aok[i], k0 + kstride + off[i], va[i]);
        load8(bp[i], bok[i], k0 + kstride + off[i], vb[i]);
      }
    }
    if (busy) {
      half8 ah[4], al[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int mt = 4 * mb + i;
        ah[i] = __builtin_bit_cast(half8, lds[st][0][(2 * mt) * 64 + lane]);
        al[i] = __builtin_bit_cast(half8, lds[st][0][(2 * mt + 1) * 64 + lane]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int nt = 8 * nb + j;
        const half8 bh = __builtin_bit_cast(half8, lds[st][1][(2 * nt) * 64 + lane]);
        const half8 bl = __builtin_bit_cast(half8, lds[st][1][(2 * nt + 1) * 64 + lane]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[i][j] = MFMA16(ah[i], bh, acc[i][j]);
          acc[i][j] = MFMA16(ah[i], bl, acc[i][j]);
          acc[i][j] = MFMA16(al[i], bh, acc[i][j]);
        }
      }
    }
    st ^= 1;   // the other stage is rewritten next step; its readers passed this barrier
  }
  if (bias_part && blockIdx.y == 0) {   // the 4 threads of a row are adjacent lanes
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float r = rsum[i];
      r += __shfl_xor(r, 1);
      r += __shfl_xor(r, 2);
      const int u = tid + 512 * i;
      if ((u & 3) == 0 && aok[i]) bias_part[(int64_t)blockIdx.z * M + m0 + (u >> 2)] = r;
    }
  }
  if (!busy) return;
  const float inv = ldexpf(1.0f, -(ea + eb));
  float* out = part + (int64_t)blockIdx.z * M * N;
  const int g4 = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + 64 * mb + 16 * i + 4 * g4 + r;
        const int n = n0 + 128 * nb + 16 * j + (lane & 15);
        if (m < M && n < N) out[(int64_t)m * N + n] = acc[i][j][r] * inv;
      }
}


// The same partial weight gradients for aligned operands (host-checked: P a
// multiple of 32, 16-B rows, operands < 2 GiB): the raw FP32 K steps land in
// LDS by buffer-form LDS-DMA, so no registers hold in-flight data. A K step
// (32 samples) is two granules of 32 KiB, A_k (256 rows of A) then B_k, and
// the granules stream through a 5-slot ring (160 KiB, all of the CU's LDS):
// while step k is multiplied, A_{k+1} and B_{k+1} are split and A_{k+2},
// B_{k+2} are landing -- B_{k+2} in A_k's slot, freed by a mid-step barrier once
// every wave holds its A_k fragments. A wave's 8 LDS-DMA pieces of a step (4 of
// A_{k+2}, then 4 of B_{k+2}) are issued one per B tile of its MFMA loop, so
// their issue cost overlaps the MFMAs.
// Piece (t, h) of a granule = 16-row tile t, half h: lane l holds row
// 16t + (l & 15), samples 8 (l >> 4) + 4h .. +3, so the two halves read by
// lane l are one MFMA fragment (row l & 15, samples 8 (l >> 4) .. +7). Rows past
// M / N read 0 (offset past num_records).
// Self split (round 5): a wave splits, in place, the fragments of the pieces it
// issued itself (granule g, tiles 2 wave + t, both halves: FP32 -> FP16 hi in
// half 0, lo in half 1), once its own vmcnt says they landed -- no barrier
// between the landing and the split; the MFMA loop reads (hi, lo) as they are.
// Every element is split once instead of by every wave that multiplies it (A
// twice, B four times): 64 instead of 192 VALU per wave and step, partials bit
// for bit those of the per-wave split. A granules add their raw values to rs
// (the bias sums: tile 2 wave + t, this lane's row and 8 samples).
// Scales: per tensor (amax_a, amax_b), or two for A (a2_row > 0: rows >=
// a2_row, whole 16-row tiles, split at amax_a2's scale and undone with it).
// The body for output tile (mtile, ntile) and K subset z of Z; subset z's
// partials go to part + z * ldpart ([M][ldo]) and bias_part + z * ldbias ([M]).
// NERF_WGRAD_ABL (timing-only study builds, results invalid): 1 no MFMAs, 2 no
// operand stream, 3 no mid-step barrier, 4 no step barrier.
constexpr int kWgRing = 5;
#ifndef NERF_WGRAD_ABL
#define NERF_WGRAD_ABL 0
#endif
__device__ __forceinline__ void wgrad_dma_body(
    uint4 (&ring)[kWgRing][32 * 64], const float* __restrict__ A, int64_t lda, int M,
    const float* __restrict__ B, int64_t ldb, int N, int64_t P, const float amax_a,
    const float amax_a2, int a2_row, const float amax_b, float* __restrict__ part,
    int64_t ldpart, float* __restrict__ bias_part, int64_t ldbias, int mtile, int ntile, int z,
    int Z, int64_t ldo, int64_t bsa, int64_t bsb) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: SGPR rsrc / M0
  const int m0 = mtile * kWgTile, n0 = ntile * kWgTile;
  const int64_t pb = (int64_t)z * 32, kstride = (int64_t)Z * 32;
  const int nsteps = pb < P ? (int)((P - pb + kstride - 1) / kstride) : 0;
  const int ngran = 2 * nsteps;
  const int ea = act_exponent(amax_a), ea2 = act_exponent(amax_a2), eb = act_exponent(amax_b);
  const float sb = ldexpf(1.0f, eb);
  // this wave's two A tiles (rows m0 + 16 (2 wave + t)): their scale
  const float sa0 = ldexpf(1.0f, m0 + 32 * wave >= a2_row ? ea2 : ea);
  const float sa1 = ldexpf(1.0f, m0 + 32 * wave + 16 >= a2_row ? ea2 : ea);

  // this wave's 4 pieces of every granule: q = 4 wave + i (tile q >> 1, half q & 1).
  // Element (r, p) of an operand: r * ld + (p >> 4) * bs + (p & 15) (bs 16:
  // feature-major rows), or Lay::rowpart(r) + (p >> 4) * bs + (p & 15) (the T16
  // layout, bs = its block stride). A K step's block offset rides in soffset,
  // the lane's row and column in voffset; num_records = the operand's extent
  // (rows past M / N read 0)
  // bs != 16: the T16 layout (Lay), rows permuted inside their 16-row groups
  const bool ta = bsa != 16, tb = bsb != 16;
  const int nbA = ta ? (int)(((P / 16 - 1) * bsa + ((M + 15) & ~15) * 16) * 4)
                     : (int)((((int64_t)M - 1) * lda + (P / 16 - 1) * bsa + 16) * 4);
  const int nbB = tb ? (int)(((P / 16 - 1) * bsb + ((N + 15) & ~15) * 16) * 4)
                     : (int)((((int64_t)N - 1) * ldb + (P / 16 - 1) * bsb + 16) * 4);
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, nbA, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)B, 0, nbB, 0x00020000);
  unsigned voA[4], voB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = 4 * wave + i, t = q >> 1, h = q & 1;
    const int col = 8 * (lane >> 4) + 4 * h;     // sample of the K step, 0 .. 31
    const int ra = m0 + 16 * t + (lane & 15), rb = n0 + 16 * t + (lane & 15);
    const int64_t rowa = ta ? Lay::rowpart(ra) : (int64_t)ra * lda;
    const int64_t rowb = tb ? Lay::rowpart(rb) : (int64_t)rb * ldb;
    voA[i] = ra < M ? (unsigned)((rowa + (col >> 4) * bsa + (col & 15)) * 4) : (unsigned)nbA;
    voB[i] = rb < N ? (unsigned)((rowb + (col >> 4) * bsb + (col & 15)) * 4) : (unsigned)nbB;
  }
  // piece I of granule g: A (g even) or B (g odd) of step g >> 1, into slot g % 5
  auto issue_piece = [&](int g, auto Ic) {
    constexpr int I = decltype(Ic)::value;
    if (g >= ngran) return;
#if NERF_WGRAD_ABL == 2
    return;
#endif
    const int64_t p0 = pb + (int64_t)(g >> 1) * kstride;   // a multiple of 32
    uint4* dst = &ring[g % kWgRing][(4 * wave + I) * 64];
    if (g & 1) {
      const int so = __builtin_amdgcn_readfirstlane((int)((p0 >> 4) * bsb * 4));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_ptr_t)dst, 16, (int)voB[I], so, 0, 0);
    } else {
      const int so = __builtin_amdgcn_readfirstlane((int)((p0 >> 4) * bsa * 4));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_ptr_t)dst, 16, (int)voA[I], so, 0, 0);
    }
  };
  auto issue = [&](int g) {
    issue_piece(g, std::integral_constant<int, 0>{});
    issue_piece(g, std::integral_constant<int, 1>{});
    issue_piece(g, std::integral_constant<int, 2>{});
    issue_piece(g, std::integral_constant<int, 3>{});
  };

  const int mb = wave & 3, nb = wave >> 2;   // wave tile: rows 64 mb.., cols 128 nb..
  const bool busy = (m0 + 64 * mb < M) && (n0 + 128 * nb < N);   // wave-uniform
  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4(0.0f);

  // a fragment's two halves (hi, lo) as the asm wrote them, 1 KiB apart. A drain
  // names every pending Raw as an in/out operand, so no copy of one can run
  // before it lands.
  struct Raw { u32x4 x, y; };
  auto read_pair = [&](unsigned addr, Raw& r) {   // addr: LDS byte address of half 0
    asm volatile("ds_read_b128 %0, %1" : "=v"(r.x) : "v"(addr) : "memory");
    asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(r.y) : "v"(addr) : "memory");
  };
  float rs[2] = {0.0f, 0.0f};
  auto split_own = [&](int g, int t, float s, bool sum) {
    u32x4* q = reinterpret_cast<u32x4*>(&ring[g % kWgRing][(2 * (2 * wave + t)) * 64 + lane]);
    const u32x4 x = q[0], y = q[64];
    Op v = __builtin_bit_cast(Op, __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7));
    if (sum) {
#pragma unroll
      for (int u = 0; u < 8; ++u) rs[t] += v[u];
    }
    split_op(v, s);
    q[0] = __builtin_bit_cast(u32x4, __builtin_shufflevector(v, v, 0, 1, 2, 3));
    q[64] = __builtin_bit_cast(u32x4, __builtin_shufflevector(v, v, 4, 5, 6, 7));
  };
  auto split_a = [&](int g, int t) { split_own(g, t, t ? sa1 : sa0, true); };
  auto split_b = [&](int g, int t) { split_own(g, t, sb, false); };

  // prologue: granules 0 .. 3 (A_0, B_0, A_1, B_1), then this wave's share of step 0
  for (int g = 0; g < 4 && g < ngran; ++g) issue(g);
  if (nsteps > 0) {
    vm_wait_n(nsteps > 1 ? 12 : 4);   // A_0 landed
    split_a(0, 0);
    split_a(0, 1);
    vm_wait_n(nsteps > 1 ? 8 : 0);    // B_0 landed
    split_b(1, 0);
    split_b(1, 1);
  }
  for (int k = 0; k < nsteps; ++k) {
    // step k's fragments were split by their owners (the prologue or step k - 1)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#if NERF_WGRAD_ABL != 4
    __builtin_amdgcn_s_barrier();   // every split visible; B_{k-1}'s slot is free
#endif
    asm volatile("" ::: "memory");
    // A_{k+2} into B_{k-1}'s slot from the start of the step; B_{k+2} into A_k's
    // slot after the mid-step barrier. This wave splits its share of A_{k+1} at
    // B tiles 4-5 and of B_{k+1} at 6-7: A lands in 1.5 steps, B in about 1.25
    // (later or earlier splits: within 1.5 %, profiles/r5_wgrad_selfsplit/)
    const int ga = 2 * k + 4, gb = 2 * k + 5;
    const bool nxt = k + 1 < nsteps, nxt2 = k + 2 < nsteps;
    if (!busy) {   // nothing to multiply: stage and split this wave's pieces
      issue(ga);
      __builtin_amdgcn_s_barrier();
      if (nxt) {
        vm_wait_n(nxt2 ? 8 : 4);
        split_a(2 * k + 2, 0);
        split_a(2 * k + 2, 1);
      }
      issue(gb);
      if (nxt) {
        vm_wait_n(nxt2 ? 8 : 0);
        split_b(2 * k + 3, 0);
        split_b(2 * k + 3, 1);
      }
      continue;
    }
    const unsigned baseA = lds_addr((const float*)&ring[(2 * k) % kWgRing][0]) + lane * 16u;
    const unsigned baseB = lds_addr((const float*)&ring[(2 * k + 1) % kWgRing][0]) + lane * 16u;
    Raw ra[4], rb[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) read_pair(baseA + (unsigned)((4 * mb + i) * 2048), ra[i]);
    read_pair(baseB + (unsigned)((8 * nb) * 2048), rb[0]);   // B tile nt = 8 nb + j
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(ra[0].x), "+v"(ra[0].y), "+v"(ra[1].x), "+v"(ra[1].y),
                   "+v"(ra[2].x), "+v"(ra[2].y), "+v"(ra[3].x), "+v"(ra[3].y),
                   "+v"(rb[0].x), "+v"(rb[0].y)
                 :
                 : "memory");
    auto tile = [&](auto Jc) {
      constexpr int j = decltype(Jc)::value;
      Raw& cur = rb[j & 1];
      if constexpr (j > 0) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(cur.x), "+v"(cur.y) : : "memory");
      const half8 bh = __builtin_bit_cast(half8, cur.x), bl = __builtin_bit_cast(half8, cur.y);
      if constexpr (j + 1 < 8) read_pair(baseB + (unsigned)((8 * nb + j + 1) * 2048), rb[(j + 1) & 1]);
#if NERF_WGRAD_ABL != 3
      if constexpr (j == 4) __builtin_amdgcn_s_barrier();
#endif
      if constexpr (j < 4) issue_piece(ga, std::integral_constant<int, j>{});
      else issue_piece(gb, std::integral_constant<int, j - 4>{});
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const half8 ah = __builtin_bit_cast(half8, ra[i].x), al = __builtin_bit_cast(half8, ra[i].y);
#if NERF_WGRAD_ABL == 1
        asm volatile("" ::"v"(ah), "v"(al), "v"(bh), "v"(bl));
#else
        acc[i][j] = MFMA16(ah, bh, acc[i][j]);
        acc[i][j] = MFMA16(ah, bl, acc[i][j]);
        acc[i][j] = MFMA16(al, bh, acc[i][j]);
#endif
      }
      if (nxt) {   // after B_{k+2} piece j - 4: A_{k+1} needs 9 (4) newer in flight, B_{k+1} 7 (0)
        if constexpr (j == 4) vm_wait_n(nxt2 ? 9 : 4);
        if constexpr (j == 6) vm_wait_n(nxt2 ? 7 : 0);
        if constexpr (j == 4 || j == 5) split_a(2 * k + 2, j - 4);
        if constexpr (j == 6 || j == 7) split_b(2 * k + 3, j - 6);
      }
    };
    tile(std::integral_constant<int, 0>{});
    tile(std::integral_constant<int, 1>{});
    tile(std::integral_constant<int, 2>{});
    tile(std::integral_constant<int, 3>{});
    tile(std::integral_constant<int, 4>{});
    tile(std::integral_constant<int, 5>{});
    tile(std::integral_constant<int, 6>{});
    tile(std::integral_constant<int, 7>{});
  }
  if (bias_part && ntile == 0) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {   // row 16 (2 wave + t) + (l & 15): lanes l, l^16, l^32, l^48
      float r = rs[t];
      r += __shfl_xor(r, 16);
      r += __shfl_xor(r, 32);
      const int row = m0 + 16 * (2 * wave + t) + lane;
      if (lane < 16 && row < M) bias_part[(int64_t)z * ldbias + row] = r;
    }
  }
  if (!busy) return;
  float* out = part + (int64_t)z * ldpart;
  const int g4 = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int mt = m0 + 64 * mb + 16 * i;   // this A tile's first row: its scale
    const float inv = ldexpf(1.0f, -((mt >= a2_row ? ea2 : ea) + eb));
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mt + 4 * g4 + r;
        const int n = n0 + 128 * nb + 16 * j + (lane & 15);
        if (m < M && n < N) out[(int64_t)m * ldo + n] = acc[i][j][r] * inv;
      }
  }
}

__global__ __launch_bounds__(kTrainThreads, 2) void x3_wgrad_dma_kernel(
    const float* __restrict__ A, int64_t lda, int M, const float* __restrict__ B, int64_t ldb,
    int N, int64_t P, const float* __restrict__ amax_a, const float* __restrict__ amax_b,
    float* __restrict__ part, float* __restrict__ bias_part) {
  __shared__ __attribute__((aligned(16))) uint4 ring[kWgRing][32 * 64];
  wgrad_dma_body(ring, A, lda, M, B, ldb, N, P, *amax_a, *amax_a, 1 << 30, *amax_b, part,
                 (int64_t)M * N, bias_part, M, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.z, N,
                 16, 16);
}

// Several weight gradients in one launch (the whole backward of a network):
// workgroup w -> (output tile t, K subset z of Z_t), the subsets of a tile
// adjacent. Z_t is per tile (nerf_x3_wgrad_batch_z): a tile whose operand rows
// are few (the heads, the 32- / 64-row remainders) streams fewer bytes per K
// step, so it takes fewer workgroups for the same finish time and the full
// tiles more. Partials: Zmax x M x N per descriptor; a tile's rows z >= Z_t
// are written as zeros (by its z = 0 workgroup) so one fixed-order sum over
// Zmax rows serves every tile.
constexpr int kWgBatchMax = 16;
constexpr int kWgTilesMax = 40;
struct WgradBatch {
  NerfWgradDesc d[kWgBatchMax];
  unsigned char t_desc[kWgTilesMax], t_m[kWgTilesMax], t_n[kWgTilesMax], t_z[kWgTilesMax];
  int t_wg_end[kWgTilesMax];   // prefix sums of Z_t
  int nt, Zmax;
};

__global__ __launch_bounds__(kTrainThreads, 2) void x3_wgrad_batch_kernel(const WgradBatch bt) {
  __shared__ __attribute__((aligned(16))) uint4 ring[kWgRing][32 * 64];
  const int w = (int)blockIdx.x;
  int t = 0;
  while (t + 1 < bt.nt && w >= bt.t_wg_end[t]) ++t;
  const int Z = bt.t_z[t];
  const int z = w - (bt.t_wg_end[t] - Z);
  const NerfWgradDesc& d = bt.d[bt.t_desc[t]];
  const int mtile = bt.t_m[t], ntile = bt.t_n[t];
  // a scale may cover two tensors' maxima (rows of two producers in one operand),
  // or A's two row blocks take one each (a2_row)
  const bool two = d.amax_a2 && d.a2_row > 0;
  const float ma = d.amax_a2 && !two ? fmaxf(*d.amax_a, *d.amax_a2) : *d.amax_a;
  const float ma2 = two ? *d.amax_a2 : ma;
  const float mb = d.amax_b2 ? fmaxf(*d.amax_b, *d.amax_b2) : *d.amax_b;
  const int64_t ldo = d.ldo ? d.ldo : d.N;
  wgrad_dma_body(ring, d.A, d.lda, d.M, d.B, d.ldb, d.N, d.P, ma, ma2, two ? d.a2_row : 1 << 30,
                 mb, d.part, d.ldpart, d.bias_part, d.ldbias, mtile, ntile, z, Z, ldo,
                 d.bsa ? d.bsa : 16, d.bsb ? d.bsb : 16);
  if (z != 0 || Z >= bt.Zmax) return;
  // zeros in the partial rows Z .. Zmax-1 of this tile (and of its bias rows)
  const int m0 = mtile * kWgTile, n0 = ntile * kWgTile;
  const int rows = min(kWgTile, d.M - m0), cols = min(kWgTile, d.N - n0);
  for (int zz = Z; zz < bt.Zmax; ++zz) {
    float* out = d.part + (int64_t)zz * d.ldpart;
    for (int i = threadIdx.x; i < rows * cols; i += kTrainThreads) {
      const int m = m0 + i / cols, n = n0 + i % cols;
      out[(int64_t)m * ldo + n] = 0.0f;
    }
    if (d.bias_part && ntile == 0)
      for (int i = threadIdx.x; i < rows; i += kTrainThreads)
        d.bias_part[(int64_t)zz * d.ldbias + m0 + i] = 0.0f;
  }
}


// Packing of the training MLP's weight matrices for x3_layer_kernel, all of a
// network in one launch (one workgroup per matrix): padded element (i, k) =
// src[rowmap[i] * ldr + colmap[k] * ldc] (0 where a map is -1), scaled by 2^sw
// with max|W| * 2^sw in [2^11, 2^12), split into FP16 (hi, lo) fragments
// [q][t][part][g][r][j] = element (16t + r, 32q + 8g + j) (nerfhip.train_mlp).
struct X3PackDesc {
  const float* src;
  int64_t ldr, ldc;
  const int* rowmap;
  const int* colmap;
  int M, K;
  uint4* out;
  int* sw;
  unsigned* amax;   // max |W| as float bits: 0 on entry, reset to 0 by the last launch
};

// A head block gathered in the packing launch: dst[i] = *(float*)table[i], or
// the scale exponent of the matrix whose amax slot table[i] & ~1 is (bit 0
// set), or 0 (table[i] == 0).
struct X3HeadGather {
  const uint64_t* table;
  float* dst;
  int64_t n;
};

// Packing in three launches over (matrix, slab) blocks: the max |W| of every
// matrix accumulated as float bits into its amax slot, then every packing
// block derives the scale exponent from it (and the head blocks are gathered),
// then a one-thread-per-matrix launch writes the exponent into sw and resets
// the amax slot for the next packing.
constexpr int kPackSlabs = 64;   // blocks per matrix (a few loads per thread: the
                                 // launches are chains of dependent map -> source loads)

__global__ __launch_bounds__(256) void x3_pack_amax_kernel(const X3PackDesc* __restrict__ descs) {
  const X3PackDesc d = descs[blockIdx.x];
  const int total = d.M * d.K;
  const int per = (total + kPackSlabs - 1) / kPackSlabs;
  const int i0 = blockIdx.y * per, i1 = min(total, i0 + per);
  float mx = 0.0f;
  // the max is order-free: walk the source along its contiguous index (a
  // transposed pack reads W column by column otherwise: one line per element)
  const bool by_row = d.ldc > d.ldr;
  for (int base = i0 + (int)threadIdx.x; base < i1; base += 4 * 256) {
    int ri[4], ck[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {   // every map load of the batch, then every source load
      const int idx = base + 256 * u;
      const int a = by_row ? idx % d.M : idx / d.K, c = by_row ? idx / d.M : idx % d.K;
      ri[u] = idx < i1 ? d.rowmap[a] : -1;
      ck[u] = idx < i1 ? d.colmap[c] : -1;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (ri[u] >= 0 && ck[u] >= 0) mx = fmaxf(mx, fabsf(d.src[ri[u] * d.ldr + ck[u] * d.ldc]));
  }
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  __shared__ float wmax[4];   // one device atomic per block (64 per matrix word)
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0)   // values >= 0: the float bits order like the floats
    atomicMax(d.amax, __float_as_uint(fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]))));
}

__device__ __forceinline__ int pack_exponent(float amax) {
  int E = 0;
  if (amax > 0.0f) (void)frexpf(amax, &E);
  return amax > 0.0f ? 12 - E : 0;   // max |W| 2^sw in [2^11, 2^12)
}

__global__ __launch_bounds__(256) void x3_pack_kernel(const X3PackDesc* __restrict__ descs, int n,
                                                     const X3HeadGather* __restrict__ heads) {
  if ((int)blockIdx.x >= n) {   // a head block's slab
    const X3HeadGather h = heads[blockIdx.x - n];
    const int64_t per = (h.n + kPackSlabs - 1) / kPackSlabs;
    const int64_t i0 = blockIdx.y * per, i1 = min(h.n, i0 + per);
    for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) {
      const uint64_t e = h.table[i];
      float v = 0.0f;
      if (e & 1u) v = (float)pack_exponent(__uint_as_float(*reinterpret_cast<const unsigned*>(e - 1u)));
      else if (e) v = *reinterpret_cast<const float*>(e);
      h.dst[i] = v;
    }
    return;
  }
  const X3PackDesc d = descs[blockIdx.x];
  const float amax = __uint_as_float(*d.amax);
  const float scale = ldexpf(1.0f, pack_exponent(amax));
  const int mt = d.M / 16;
  const int groups = (d.K / 32) * mt * 64;   // (q, t, lane) -> 8 halfs hi + 8 halfs lo
  const int per = (groups + kPackSlabs - 1) / kPackSlabs;
  const int g0 = blockIdx.y * per, g1 = min(groups, g0 + per);
  for (int gi = g0 + (int)threadIdx.x; gi < g1; gi += 256) {
    const int lane = gi & 63, qt = gi >> 6;
    const int q = qt / mt, t = qt - q * mt;
    const int row = 16 * t + (lane & 15), k0 = 32 * q + 8 * (lane >> 4);
    const int ri = d.rowmap[row];
    half8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ck = d.colmap[k0 + j];
      const float v = (ri >= 0 && ck >= 0) ? d.src[ri * d.ldr + ck * d.ldc] * scale : 0.0f;
      const _Float16 h = (_Float16)v;
      hi[j] = h;
      lo[j] = (_Float16)(v - (float)h);
    }
    const int blk = (q * mt + t) * 2;
    d.out[blk * 64 + lane] = __builtin_bit_cast(uint4, hi);
    d.out[(blk + 1) * 64 + lane] = __builtin_bit_cast(uint4, lo);
  }
}

__global__ void x3_pack_scale_kernel(const X3PackDesc* __restrict__ descs, int n) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m < n) {
    *descs[m].sw = pack_exponent(__uint_as_float(*descs[m].amax));
    *descs[m].amax = 0u;
  }
}

}  // namespace nerfhip

using namespace nerfhip;

extern "C" int nerf_mlp_forward_x3(const float* w_slices, const float* w_head, const float* rays_o,
                                   const float* rays_d, const float* z, int64_t z_stride,
                                   int64_t n, int S, float* raw, nerf_stream_t stream) {
  NERF_REQUIRE(w_slices && w_head && rays_o && rays_d && z && raw,
               "nerf_mlp_forward_x3: null pointer");
  NERF_REQUIRE(n >= 0 && S >= 1 && z_stride >= 0, "nerf_mlp_forward_x3: bad size");
  NERF_REQUIRE(((uintptr_t)w_slices & 15) == 0 && ((uintptr_t)w_head & 15) == 0 &&
                   ((uintptr_t)raw & 15) == 0,
               "nerf_mlp_forward_x3: weights/raw must be 16-byte aligned");
  const int64_t total = n * S;
  if (total == 0) return 0;
  const int64_t blocks = cdiv(total, kX3Tile);
  NERF_REQUIRE(blocks < (1ll << 31), "nerf_mlp_forward_x3: too many samples for one launch");
  // persistent: one workgroup per CU (the ring and head take 140 KiB of the 160 KiB LDS)
  const int n_cu = stream_cu_count(stream);
  const int64_t grid = blocks < n_cu ? blocks : n_cu;
  hipLaunchKernelGGL(mlp_x3_kernel<false>, dim3((unsigned)grid), dim3(kX3Threads), 0,
                     as_stream(stream), (const float4*)w_slices, w_head, rays_o, rays_d, z,
                     z_stride, total, S, (float4*)raw, nullptr, nullptr);
  return check_launch("mlp_x3_kernel");
}

extern "C" int nerf_mlp_forward_x3_clock(const float* w_slices, const float* w_head,
                                         const float* rays_o, const float* rays_d, const float* z,
                                         int64_t z_stride, int64_t n, int S, float* raw,
                                         unsigned long long* clk, int64_t clk_len,
                                         unsigned long long* trace, nerf_stream_t stream) {
  NERF_REQUIRE(w_slices && w_head && rays_o && rays_d && z && raw && clk && trace,
               "nerf_mlp_forward_x3_clock: null pointer");
  NERF_REQUIRE(n > 0 && S >= 1 && z_stride >= 0, "nerf_mlp_forward_x3_clock: bad size");
  NERF_REQUIRE(((uintptr_t)w_slices & 15) == 0 && ((uintptr_t)w_head & 15) == 0 &&
                   ((uintptr_t)raw & 15) == 0 && ((uintptr_t)clk & 31) == 0,
               "nerf_mlp_forward_x3_clock: weights/raw/clk misaligned");
  const int64_t blocks = cdiv(n * S, kX3Tile);
  const int n_cu = stream_cu_count(stream);
  const int64_t grid = blocks < n_cu ? blocks : n_cu;
  NERF_REQUIRE(clk_len >= 4 * grid, "nerf_mlp_forward_x3_clock: clk holds < 4 per workgroup");
  hipLaunchKernelGGL(mlp_x3_clock_kernel, dim3((unsigned)grid), dim3(kX3Threads), 0,
                     as_stream(stream), (const float4*)w_slices, w_head, rays_o, rays_d, z,
                     z_stride, n * S, S, (float4*)raw, clk, trace);
  return check_launch("mlp_x3_clock_kernel");
}

extern "C" int nerf_mlp_train_forward_x3(const float* w_slices, const float* w_head,
                                         const float* pts, const float* dirs, const float* zero,
                                         int64_t P, const NerfX3TrainOut* out, float* raw,
                                         nerf_stream_t stream) {
  return nerf_mlp_train_forward_x3_rays(w_slices, w_head, pts, dirs, zero, 0, P, 1, out, raw,
                                        stream);
}

// the training kernels' output layout (Lay): feature-major rows need ld >= P and
// 256 rows within 2 GiB; T16 (bs > 0) needs whole 16-row groups per block
// (bs % 256 == 0) and the buffer within 2 GiB. 32-bit offsets either way.
static bool lay_ok(int64_t ld, int64_t bs, int64_t P) {
  if (bs == 0) return ld >= P && (int64_t)256 * ld * 4 < (1ll << 31);
  const int64_t nblk = cdiv(P, kX3Tile) * 8;
  return bs > 0 && bs % 256 == 0 && nblk * bs * 4 < (1ll << 31);
}
static Lay make_lay(int64_t ld, int64_t bs, int64_t P) {
  Lay L;
  L.ld = bs ? 16 : ld;
  L.bs = bs;
  L.nblk = cdiv(P, kX3Tile) * 8;
  return L;
}

extern "C" int nerf_mlp_train_forward_x3_rays(const float* w_slices, const float* w_head,
                                              const float* rays_o, const float* rays_d,
                                              const float* z, int64_t z_stride, int64_t n, int S,
                                              const NerfX3TrainOut* out, float* raw,
                                              nerf_stream_t stream) {
  NERF_REQUIRE(w_slices && w_head && rays_o && rays_d && z && out && raw && out->amax,
               "nerf_mlp_train_forward_x3: null pointer");
  NERF_REQUIRE(n >= 0 && S >= 1 && z_stride >= 0, "nerf_mlp_train_forward_x3: bad size");
  const int64_t P = n * S;
  NERF_REQUIRE(lay_ok(out->ld, out->bs, P), "nerf_mlp_train_forward_x3: bad layout");
  for (int i = 0; i < 12; ++i)   // act[8] (the feature rows) may be null: not stored
    NERF_REQUIRE(i == 8 || out->act[i] != nullptr, "nerf_mlp_train_forward_x3: null output rows");
  for (int i = 0; i < 9; ++i)
    NERF_REQUIRE(out->bits[i] != nullptr, "nerf_mlp_train_forward_x3: null relu bits");

  NERF_REQUIRE(((uintptr_t)w_slices & 15) == 0 && ((uintptr_t)w_head & 15) == 0 &&
                   ((uintptr_t)raw & 15) == 0,
               "nerf_mlp_train_forward_x3: weights/raw must be 16-byte aligned");
  if (P == 0) return 0;
  const int64_t blocks = cdiv(P, kX3Tile);
  NERF_REQUIRE(blocks < (1ll << 31), "nerf_mlp_train_forward_x3: too many samples");
  const int n_cu = stream_cu_count(stream);
  const int64_t grid = blocks < n_cu ? blocks : n_cu;
  X3TrainOut to;
  for (int i = 0; i < 12; ++i) to.act[i] = out->act[i];
  for (int i = 0; i < 9; ++i) to.bits[i] = out->bits[i];
  to.amax = out->amax;
  to.lay = make_lay(out->ld, out->bs, P);
  if (out->bs)
    hipLaunchKernelGGL(mlp_x3_train_kernel<true>, dim3((unsigned)grid), dim3(kX3Threads), 0,
                       as_stream(stream), (const float4*)w_slices, w_head, rays_o, rays_d, z,
                       z_stride, P, S, (float4*)raw, to);
  else
    hipLaunchKernelGGL(mlp_x3_train_kernel<false>, dim3((unsigned)grid), dim3(kX3Threads), 0,
                       as_stream(stream), (const float4*)w_slices, w_head, rays_o, rays_d, z,
                       z_stride, P, S, (float4*)raw, to);
  return check_launch("mlp_x3_train_kernel");
}

extern "C" int nerf_mlp_train_backward_x3(const float* w_slices, const float* w_head, int64_t P,
                                          int with_enc, const NerfX3BwdIO* io,
                                          nerf_stream_t stream) {
  NERF_REQUIRE(w_slices && w_head && io && io->d_raw && io->dmax,
               "nerf_mlp_train_backward_x3: null pointer");
  NERF_REQUIRE(P >= 0 && lay_ok(io->ld, io->bs, P), "nerf_mlp_train_backward_x3: bad layout");
  for (int i = 0; i < 10; ++i)   // d[8] (d feature) does not exist: the feature layer is folded
    NERF_REQUIRE((i == 8) == (io->d[i] == nullptr), "nerf_mlp_train_backward_x3: null output rows"
                 " (or d[8] set: the folded backward has no d feature)");
  if (with_enc)
    NERF_REQUIRE(io->d[10] && io->d[11], "nerf_mlp_train_backward_x3: null encoding rows");
  for (int i = 0; i < 9; ++i)
    NERF_REQUIRE(io->bits[i] != nullptr, "nerf_mlp_train_backward_x3: null relu bits");

  NERF_REQUIRE(((uintptr_t)w_slices & 15) == 0 && ((uintptr_t)w_head & 15) == 0 &&
                   ((uintptr_t)io->d_raw & 15) == 0,
               "nerf_mlp_train_backward_x3: weights/d_raw must be 16-byte aligned");
  if (P == 0) return 0;
  const int64_t blocks = cdiv(P, kX3Tile);
  NERF_REQUIRE(blocks < (1ll << 31), "nerf_mlp_train_backward_x3: too many samples");
  const int n_cu = stream_cu_count(stream);
  const int64_t grid = blocks < n_cu ? blocks : n_cu;
  X3BwdIO b;
  b.d_raw = (const float4*)io->d_raw;
  for (int i = 0; i < 9; ++i) b.bits[i] = io->bits[i];
  for (int i = 0; i < 12; ++i) b.d[i] = io->d[i];
  b.dmax = io->dmax;
  b.lay = make_lay(io->ld, io->bs, P);
  b.d_raw_t = io->d_raw_t;
  auto* k = with_enc ? (io->bs ? mlp_x3_bwd_kernel<true, true> : mlp_x3_bwd_kernel<true, false>)
                     : (io->bs ? mlp_x3_bwd_kernel<false, true> : mlp_x3_bwd_kernel<false, false>);
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(kX3Threads), 0, as_stream(stream),
                     (const float4*)w_slices, w_head, P, b);
  return check_launch("mlp_x3_bwd_kernel");
}

extern "C" int nerf_mlp_forward_x3_list(const float* w_slices, const float* w_head,
                                        const float* rays_o, const float* rays_d, const float* z,
                                        int64_t z_stride, int S, const int* list,
                                        const int* count, int64_t max_count, float* raw,
                                        nerf_stream_t stream) {
  NERF_REQUIRE(w_slices && w_head && rays_o && rays_d && z && raw && list && count,
               "nerf_mlp_forward_x3_list: null pointer");
  NERF_REQUIRE(S >= 1 && z_stride >= 0 && max_count >= 0, "nerf_mlp_forward_x3_list: bad size");
  NERF_REQUIRE(((uintptr_t)w_slices & 15) == 0 && ((uintptr_t)w_head & 15) == 0 &&
                   ((uintptr_t)raw & 15) == 0,
               "nerf_mlp_forward_x3_list: weights/raw must be 16-byte aligned");
  if (max_count == 0) return 0;
  const int64_t blocks = cdiv(max_count, kX3Tile);
  NERF_REQUIRE(blocks < (1ll << 31), "nerf_mlp_forward_x3_list: too many samples");
  const int n_cu = stream_cu_count(stream);
  const int64_t grid = blocks < n_cu ? blocks : n_cu;   // persistent: the count is device-side
  hipLaunchKernelGGL(mlp_x3_kernel<true>, dim3((unsigned)grid), dim3(kX3Threads), 0,
                     as_stream(stream), (const float4*)w_slices, w_head, rays_o, rays_d, z,
                     z_stride, (int64_t)0, S, (float4*)raw, list, count);
  return check_launch("mlp_x3_kernel");
}

template <int MT, int NK, int EPI>
static int launch_layer(const float* w, const int* sw, const float* bias, const float* B,
                        int64_t ldb, const float* mask, int64_t ldm, const float* ru,
                        const float* rw, float* C, int64_t ldc, int64_t P, float* amax_out,
                        unsigned short* bits_out, const unsigned short* bits_in,
                        const float* head_w, const float* head_b, int n_head, float* head_out,
                        int head_col, nerf_stream_t stream) {
  // persistent: at most one workgroup per CU (the ring takes 64-128 KiB of LDS)
  const int64_t tiles = cdiv(P, kTrainTile);
  const int n_cu = stream_cu_count(stream);
  hipLaunchKernelGGL((x3_layer_kernel<MT, NK, EPI>), dim3((unsigned)(tiles < n_cu ? tiles : n_cu)),
                     dim3(kTrainThreads), 0, as_stream(stream), (const uint4*)w, sw, bias, B,
                     ldb, mask, ldm, ru, rw, C, ldc, P, amax_out, bits_out, bits_in, head_w,
                     head_b, n_head, head_out, head_col);
  return check_launch("x3_layer_kernel");
}

extern "C" int nerf_x3_layer(const float* w_packed, const int* w_scale, int m_tiles, int k_steps,
                             const float* bias, const float* B, int64_t ldb, const float* mask,
                             int64_t ldm, const float* ru, const float* rw, int relu, float* C,
                             int64_t ldc, int64_t P, float* amax_out, nerf_stream_t stream) {
  return nerf_x3_layer_ex(w_packed, w_scale, m_tiles, k_steps, bias, B, ldb, mask, ldm, ru, rw,
                          relu, C, ldc, P, amax_out, nullptr, nullptr, nullptr, nullptr, 0,
                          nullptr, 0, stream);
}

extern "C" int nerf_x3_layer_ex(const float* w_packed, const int* w_scale, int m_tiles,
                                int k_steps, const float* bias, const float* B, int64_t ldb,
                                const float* mask, int64_t ldm, const float* ru, const float* rw,
                                int relu, float* C, int64_t ldc, int64_t P, float* amax_out,
                                unsigned short* relu_bits, const unsigned short* mask_bits,
                                const float* head_w, const float* head_b, int n_head,
                                float* head_out, int head_col, nerf_stream_t stream) {
  NERF_REQUIRE(!head_out || (head_w && head_b && n_head >= 1 && n_head <= 3 && head_col >= 0 &&
                             head_col + n_head <= 4 && ((uintptr_t)head_w & 15) == 0),
               "nerf_x3_layer: head needs 16-byte aligned head_w [n_head][16 m_tiles], head_b, "
               "1 <= n_head <= 3 columns inside [0, 4)");
  NERF_REQUIRE(w_packed && w_scale && B && C, "nerf_x3_layer: null pointer");
  NERF_REQUIRE(!(mask && mask_bits), "nerf_x3_layer: mask and mask_bits are exclusive");
  NERF_REQUIRE(!relu_bits || relu, "nerf_x3_layer: relu_bits needs relu");
  NERF_REQUIRE((((uintptr_t)relu_bits) | ((uintptr_t)mask_bits)) % 2 == 0,
               "nerf_x3_layer: bit words must be 2-byte aligned");
  NERF_REQUIRE((ru == nullptr) == (rw == nullptr), "nerf_x3_layer: ru and rw go together");
  NERF_REQUIRE(P >= 0 && ldb >= P && ldc >= P && (!mask || ldm >= P), "nerf_x3_layer: bad size");
  NERF_REQUIRE(((uintptr_t)w_packed & 15) == 0, "nerf_x3_layer: packed W must be 16-byte aligned");
  NERF_REQUIRE(cdiv(P, kTrainTile) < (1ll << 31), "nerf_x3_layer: too many samples");
  NERF_REQUIRE(128ll * k_steps * ldb < (1ll << 31) && 64ll * m_tiles * ldc < (1ll << 31) &&
                   (!mask || 64ll * m_tiles * ldm < (1ll << 31)),
               "nerf_x3_layer: an operand spans 2 GiB or more (32-bit buffer offsets)");
  if (P == 0) return 0;
  const int epi = (bias ? kEpiBias : 0) | (relu ? kEpiRelu : 0) | (mask ? kEpiMask : 0) |
                  (ru ? kEpiRank1 : 0) | (mask_bits ? kEpiMaskBits : 0) |
                  (relu_bits ? kEpiOutBits : 0) | (head_out ? kEpiHead : 0);
#define NERF_LAYER_CASE(MT, NK, EPI)                                                          \
  if (m_tiles == MT && k_steps == NK && epi == (EPI))                                         \
    return launch_layer<MT, NK, (EPI)>(w_packed, w_scale, bias, B, ldb, mask, ldm, ru, rw, C, \
                                       ldc, P, amax_out, relu_bits, mask_bits, head_w, head_b,   \
                                       n_head, head_out, head_col, stream);
  // forward layers (bias + ReLU; the feature layer without ReLU)
  NERF_LAYER_CASE(16, 2, kEpiBias | kEpiRelu) NERF_LAYER_CASE(16, 8, kEpiBias | kEpiRelu)
  NERF_LAYER_CASE(16, 10, kEpiBias | kEpiRelu) NERF_LAYER_CASE(8, 9, kEpiBias | kEpiRelu)
  NERF_LAYER_CASE(16, 8, kEpiBias)
  // backward layers (ReLU mask; + the alpha head's rank-1 term into d h7)
  NERF_LAYER_CASE(16, 4, 0) NERF_LAYER_CASE(16, 8, kEpiMask)
  NERF_LAYER_CASE(16, 8, kEpiMask | kEpiRank1) NERF_LAYER_CASE(4, 8, 0)
  // the training MLP's mask path: forward layers write their ReLU bits, the
  // dgrad layers read them (32 B per sample and layer instead of 1 KiB)
  NERF_LAYER_CASE(16, 2, kEpiBias | kEpiRelu | kEpiOutBits)
  NERF_LAYER_CASE(16, 8, kEpiBias | kEpiRelu | kEpiOutBits)
  NERF_LAYER_CASE(16, 10, kEpiBias | kEpiRelu | kEpiOutBits)
  NERF_LAYER_CASE(16, 8, kEpiMaskBits) NERF_LAYER_CASE(16, 8, kEpiMaskBits | kEpiRank1)
  // + the heads: alpha on layer 7, rgb on the views layer (which also writes its
  // bits for the d_hv launch (8, 1, mask bits))
  NERF_LAYER_CASE(16, 8, kEpiBias | kEpiRelu | kEpiOutBits | kEpiHead)
  NERF_LAYER_CASE(8, 9, kEpiBias | kEpiRelu | kEpiOutBits | kEpiHead)
  NERF_LAYER_CASE(8, 1, kEpiMaskBits)
  // every term at once (tests)
  NERF_LAYER_CASE(16, 8, kEpiBias | kEpiRelu | kEpiMask | kEpiRank1)
#undef NERF_LAYER_CASE
  return fail(NERF_E_UNSUPPORTED, "nerf_x3_layer: unsupported (m_tiles, k_steps, epilogue)");
}

static bool wgrad_dma_ok(const float* A, int64_t lda, int M, const float* B, int64_t ldb, int N,
                         int64_t P, int64_t bsa = 16, int64_t bsb = 16) {
  const int64_t ea = bsa != 16 ? (P / 16 - 1) * bsa + ((M + 15) & ~15) * 16   // operand extents
                               : ((int64_t)M - 1) * lda + (P / 16 - 1) * bsa + 16;
  const int64_t eb = bsb != 16 ? (P / 16 - 1) * bsb + ((N + 15) & ~15) * 16
                               : ((int64_t)N - 1) * ldb + (P / 16 - 1) * bsb + 16;
  return P % 32 == 0 && lda % 4 == 0 && ldb % 4 == 0 && bsa % 4 == 0 && bsb % 4 == 0 &&
         ((((uintptr_t)A) | ((uintptr_t)B)) & 15) == 0 &&
         ea * 4 < ((int64_t)1 << 31) && eb * 4 < ((int64_t)1 << 31);
}

extern "C" int nerf_x3_wgrad(const float* A, int64_t lda, int M, const float* B, int64_t ldb,
                             int N, int64_t P, int64_t chunk, const float* amax_a,
                             const float* amax_b, float* part, float* bias_part,
                             nerf_stream_t stream) {
  NERF_REQUIRE(A && B && amax_a && amax_b && part, "nerf_x3_wgrad: null pointer");
  NERF_REQUIRE(M > 0 && N > 0 && P >= 0 && lda >= P && ldb >= P && chunk > 0 && chunk % 32 == 0,
               "nerf_x3_wgrad: bad size");
  const int64_t chunks = cdiv(P, chunk);
  if (chunks == 0) return 0;
  NERF_REQUIRE(chunks < 65536, "nerf_x3_wgrad: too many chunks");
  const dim3 grid((unsigned)cdiv(M, kWgTile), (unsigned)cdiv(N, kWgTile), (unsigned)chunks);
  const bool dma = wgrad_dma_ok(A, lda, M, B, ldb, N, P);
  if (dma) {
    hipLaunchKernelGGL(x3_wgrad_dma_kernel, grid, dim3(kTrainThreads), 0, as_stream(stream), A,
                       lda, M, B, ldb, N, P, amax_a, amax_b, part, bias_part);
    return check_launch("x3_wgrad_dma_kernel");
  }
  hipLaunchKernelGGL(x3_wgrad_kernel, grid, dim3(kTrainThreads), 0, as_stream(stream), A, lda, M,
                     B, ldb, N, P, chunk, amax_a, amax_b, part, bias_part);
  return check_launch("x3_wgrad_kernel");
}


extern "C" int nerf_x3_wgrad_batch_z(const NerfWgradDesc* descs, int n, const int* tile_chunks,
                                     int zmax, nerf_stream_t stream) {
  NERF_REQUIRE(descs && tile_chunks && n >= 1 && n <= kWgBatchMax && zmax >= 1 && zmax < 65536,
               "nerf_x3_wgrad_batch: bad arguments");
  WgradBatch bt;
  int nt = 0, wgs = 0;
  for (int k = 0; k < n; ++k) {
    const NerfWgradDesc& d = descs[k];
    const int64_t ldo = d.ldo ? d.ldo : d.N;
    const int64_t bsa = d.bsa ? d.bsa : 16, bsb = d.bsb ? d.bsb : 16;
    // feature-major rows hold every sample (ld >= P); in the block layout a
    // block holds every row (bs >= 16 rows, ld = 16)
    NERF_REQUIRE(d.A && d.B && d.amax_a && d.amax_b && d.part && d.M > 0 && d.N > 0 &&
                     d.P >= 0 && (bsa == 16 ? d.lda >= d.P : bsa % 256 == 0 && bsa >= 16 * d.M) &&
                     (bsb == 16 ? d.ldb >= d.P : bsb % 256 == 0 && bsb >= 16 * d.N) && ldo >= d.N &&
                     d.ldpart >= (int64_t)(d.M - 1) * ldo + d.N &&
                     (!d.bias_part || d.ldbias >= d.M) &&
                     (d.a2_row == 0 || (d.amax_a2 && d.a2_row > 0 && d.a2_row % 16 == 0 &&
                                        d.a2_row < d.M)),
                 "nerf_x3_wgrad_batch: bad descriptor");
    NERF_REQUIRE(wgrad_dma_ok(d.A, d.lda, d.M, d.B, d.ldb, d.N, d.P, bsa, bsb),
                 "nerf_x3_wgrad_batch: operands must be aligned (P % 32 == 0, 16-B rows, < 2 GiB)");
    bt.d[k] = d;
    const int mt = (int)cdiv(d.M, kWgTile), ntl = (int)cdiv(d.N, kWgTile);
    for (int j = 0; j < ntl; ++j)       // tile order: descriptor, then N tile, then M tile
      for (int i = 0; i < mt; ++i) {
        NERF_REQUIRE(nt < kWgTilesMax, "nerf_x3_wgrad_batch: too many tiles");
        const int Z = tile_chunks[nt];
        NERF_REQUIRE(Z >= 1 && Z <= zmax && Z < 256, "nerf_x3_wgrad_batch: bad tile chunks");
        bt.t_desc[nt] = (unsigned char)k;
        bt.t_m[nt] = (unsigned char)i;
        bt.t_n[nt] = (unsigned char)j;
        bt.t_z[nt] = (unsigned char)Z;
        wgs += Z;
        bt.t_wg_end[nt] = wgs;
        ++nt;
      }
  }
  bt.nt = nt;
  bt.Zmax = zmax;
  hipLaunchKernelGGL(x3_wgrad_batch_kernel, dim3((unsigned)wgs), dim3(kTrainThreads), 0,
                     as_stream(stream), bt);
  return check_launch("x3_wgrad_batch_kernel");
}

extern "C" int nerf_x3_wgrad_batch(const NerfWgradDesc* descs, int n, int chunks,
                                   nerf_stream_t stream) {
  NERF_REQUIRE(descs && n >= 1 && n <= kWgBatchMax && chunks >= 1 && chunks < 256,
               "nerf_x3_wgrad_batch: bad arguments");
  int zs[kWgTilesMax];
  for (int i = 0; i < kWgTilesMax; ++i) zs[i] = chunks;
  return nerf_x3_wgrad_batch_z(descs, n, zs, chunks, stream);
}

extern "C" int nerf_x3_pack(const void* descs, int n, const void* heads, int n_heads,
                            nerf_stream_t stream) {
  NERF_REQUIRE(descs && n > 0 && n < 65536 && n_heads >= 0 && n_heads < 256 &&
                   (heads || n_heads == 0),
               "nerf_x3_pack: bad arguments");
  const X3PackDesc* d = (const X3PackDesc*)descs;
  hipLaunchKernelGGL(x3_pack_amax_kernel, dim3((unsigned)n, kPackSlabs), dim3(256), 0,
                     as_stream(stream), d);
  hipLaunchKernelGGL(x3_pack_kernel, dim3((unsigned)(n + n_heads), kPackSlabs), dim3(256), 0,
                     as_stream(stream), d, n, (const X3HeadGather*)heads);
  hipLaunchKernelGGL(x3_pack_scale_kernel, dim3((unsigned)cdiv(n, 64)), dim3(64), 0,
                     as_stream(stream), d, n);
  return check_launch("x3_pack_kernel");
}
