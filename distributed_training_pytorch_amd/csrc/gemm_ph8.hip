// Eight-phase LDS-DMA bf16 GEMM for gfx950 (CDNA4): the wide-MLP layer GEMMs
// (forward x W^T, input gradient dz W, weight gradient dz^T h) with the fused
// Linear epilogues of gemm_epi.h.  Same contract as dtp_gemm's 256x256 kernels
// (csrc/gemm.hip): C[M,N] (+)= epi(alpha * A(m,:) . B(n,:)).
//
// Why a second 256x256 kernel: the two-buffer kernel of gemm.hip issues tile t+1's
// LDS-DMA, runs tile t, then drains vmcnt(0) + barrier, so every K-tile waits out a
// full DMA round trip that only one tile of MFMA work covers (profiles/gemm_r1_fast:
// a third of wave time parked in s_waitcnt / s_barrier, 1.19 PF at 4096^3 vs
// hipBLASLt 1.57).  Here the staging granule is a quarter tile and the wait is
// counted, so three quarter tiles stay in flight across every barrier:
//
//  * block tile 256 x 256 x 64, 8 waves as 2 (M) x 4 (N).  Wave (wr, wc) owns the
//    rows {wr*64 + [0,64)} and {128 + wr*64 + [0,64)} and the columns
//    {wc*32 + [0,32)} and {128 + wc*32 + [0,32)}: 8 x 4 fragments of
//    v_mfma_f32_16x16x32_bf16 (128 accumulators), split into four quadrants
//    (qm, qn) of 4 x 2 fragments.  Quadrant qm of every wave lives in the operand
//    PART A_qm = tile rows [128 qm, +128), quadrant qn in B_qn = tile columns
//    [128 qn, +128): each of the four parts is read in exactly one phase per tile.
//  * one K-tile = 4 phases, one quadrant (16 MFMAs = 256 matrix cycles) each.  The
//    simple schedule (variant 2) reads 12 / 4 / 8 / 0 fragments per phase:
//        phase 0: read A0 + B0 fragments, MFMA quadrant (0,0), DMA A0 of tile u+1
//        phase 1: read B1,               MFMA (0,1),            DMA B1 of tile u+1
//        phase 2: read A1,               MFMA (1,1),            DMA A1 of tile u+1
//        phase 3: (registers only),      MFMA (1,0),            DMA B0 of tile u+2
//    The default (balanced) schedule reads 8 / 4 / 8 / 4: phase 3 pre-reads the next
//    tile's first B part into the register set phase 2 released, so a tile's two B
//    quadrants alternate between register sets and the K loop runs tiles in pairs.
//    Registers: 128 accumulators + A quadrant (32) + both B quadrants (32); the lane
//    address state is made opaque once per tile so LICM cannot hoist every phase's
//    addresses into live registers (it spilled the balanced instances).
//  * split-K (few output tiles, long K: launch_ph8 with splitk > 1): each block runs
//    a K-slice and stores raw f32 partials to a workspace; splitk_reduce_kernel sums
//    the slices and applies the epilogue.
//  * LDS: 2 K-tile buffers x 4 parts x 16 KiB = 128 KiB, plus one 16 KiB sink
//    for the DMA slots past the last tile (so every phase issues exactly one part
//    and the wait count never changes).
//  * every phase: [fragment reads] [one part's DMA: 2 global_load_lds_dwordx4 per
//    wave] s_waitcnt vmcnt(6) | s_barrier | lgkmcnt(0), 16 MFMAs at s_setprio 1 |
//    s_barrier.  vmcnt(6) leaves the three youngest parts in flight and retires
//    the part read in the NEXT phase (staged 4 or 5 phases before its read);
//    a part is restaged >= 3 phases after its last read (WAR).
//  * stagger: waves 4-7 (the second wave of each SIMD) run one barrier behind, so
//    on every SIMD one wave's fragment reads and DMA issue overlap its partner's
//    MFMA segment (cdna_hip_programming.md §5 "The 256² 8-phase template",
//    MI355X_MICROARCH.md "Two waves per SIMD").  With the wait placed before the
//    first barrier of a phase, a read one phase later is ordered for both groups.
//  * LDS images (the DMA writes lane-linear; the bank swizzles ride on the DMA
//    SOURCE address and the matching XOR on the read, fswz(x) = (x&3)|((x>>1)&4)):
//      K-contiguous operand: [128 rows][8 x 16-B chunks], chunk c of row r at
//        c ^ fswz(r); a fragment is one conflict-free ds_read_b128;
//      M/N-contiguous operand: [64 k][128 columns] (256-B k-rows), 32-B granule g
//        of k-row k at g ^ fswz(k); a fragment is two ds_read_b64_tr_b16 whose
//        32-lane halves touch 8 distinct 32-B windows of the bank row.
// Preconditions (dtp_gemm checks them): K % 64 == 0, 16-byte aligned rows, a
// transposed operand's M/N a multiple of 8.  Rows/columns past M/N are clamped on
// load and never stored.
#include "gemm_epi.h"

namespace dtp {
namespace gemm {
namespace ph8 {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;

constexpr int kThreads = 512;
constexpr int kPart = 128 * 64 * 2;      // one operand part of one K-tile (16 KiB)
constexpr int kBuf = 4 * kPart;          // parts A0, A1, B0, B1
constexpr int kSink = 2 * kBuf;          // DMA sink for the slots past the last K-tile
constexpr int kLds = kSink + kPart;      // 144 KiB
static_assert(8 * kEpiWaveFloats * 4 <= kLds, "epilogue staging must fit the operand LDS");

DTP_DEV int fswz(int x) { return (x & 3) | ((x >> 1) & 4); }

// Per-lane DMA source offsets (bytes, relative to the block's first operand row /
// column r0; the uniform part of the address -- operand base, r0, K-tile -- rides
// in SGPRs: global_load_lds's saddr form) of the two wave-instructions that fill
// part p (operand rows, or columns, [r0 + 128 p, +128) of a K-tile): instruction i
// of wave w fills part bytes [(8 i + w) KiB, +1 KiB).
template <bool TRANS>
DTP_DEV void part_sources(uint32_t (&off)[2][2], long long ld, int r0, int R, int wave, int lane) {
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if constexpr (!TRANS) {  // 8 rows x 128 B per instruction
        const int row = (8 * i + wave) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ fswz(row);
        const int rr = min(r0 + 128 * p + row, R - 1) - r0;
        off[p][i] = static_cast<uint32_t>((static_cast<long long>(rr) * ld + c * 8) * 2);
      } else {  // 4 k-rows x 256 B per instruction
        const int k = (8 * i + wave) * 4 + (lane >> 4);
        const int c = (lane & 15) ^ (fswz(k) << 1);
        const int col = min(r0 + 128 * p + c * 8, R - 8) - r0;
        off[p][i] = static_cast<uint32_t>((static_cast<long long>(k) * ld + col) * 2);
      }
    }
}

// Byte offsets of this lane's fragment reads inside a part.  Row image: off[ks]
// for k-step ks, fragment f (16 rows) adds 2048 f.  k-major image: off[f] for
// fragment f (16 columns) at k-step 0; k-step 1 adds 32 k-rows (8192 B), the upper
// 4 k of a lane's 8 another 4 k-rows (1024 B).
template <bool TRANS, int NF>
DTP_DEV void part_offsets(int (&off)[TRANS ? NF : 2], int rb, int lane) {
  const int lr = lane & 15, lg = lane >> 4;
  if constexpr (!TRANS) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) off[ks] = ((rb + lr) * 8 + ((4 * ks + lg) ^ fswz(lr))) * 16;
  } else {
    // lane 4q+p of group lg supplies k-row 8 lg + q (+ 32 ks, + 4), columns 4p..4p+3
    const int q = lr >> 2, p = lr & 3, sw = q | ((lg & 1) << 2);
#pragma unroll
    for (int f = 0; f < NF; ++f) off[f] = (8 * lg + q) * 256 + ((((rb + 16 * f) >> 4) ^ sw) << 5) + 8 * p;
  }
}

template <bool TRANS>
DTP_DEV bf16x8 frag(const char* part, const int* off, int f, int ks) {
  if constexpr (!TRANS) {
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(part + off[ks] + f * 2048));
  } else {
    // inline asm: hipcc treats the ds_read_tr16 builtin as possibly aliasing the
    // in-flight LDS-DMA and drains vmcnt(0) before it, which would empty the DMA
    // pipeline every phase.  The reads complete under mid()'s lgkmcnt(0), pinned by
    // its sched_barrier (cdna_hip_programming.md §5.4 rule 18).
    const uint32_t p = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)(part + off[f] + ks * 8192)));
    bf16x4 lo, hi;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(p));
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:1024" : "=v"(hi) : "v"(p));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

DTP_DEV void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// PERSIST: one workgroup per CU walks the tiles t = blockIdx.x + i * gridDim.x; after a
// tile's K loop it issues the NEXT tile's five prologue parts (buffer 0 and part 3 of
// buffer 1) before its own epilogue, which stages 16-row passes in the LDS gap between
// them ([64 KiB, 98 KiB)), so the next tile's operand fill runs under this tile's
// write-back instead of after a new workgroup's start (profiles/r4_gemm: ~3 points of
// per-tile cost).  Balanced schedule only (its prologue leaves that gap free).
template <bool TA, bool TB, bool BAL, bool SPLIT, bool PERSIST = false>
__global__ __launch_bounds__(kThreads) void gemm_ph8_kernel(DtpGemmArgs a) {
  static_assert(!PERSIST || (BAL && !SPLIT), "the persistent walk runs the balanced, unsplit schedule");
  __shared__ __align__(16) char lds[kLds];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int ntiles = PERSIST ? ((a.M + 255) / 256) * ((a.N + 255) / 256) : 0;
  int tcur = blockIdx.x;
  if (PERSIST && tcur >= ntiles) return;  // the grid is rounded up to a multiple of 8 (whole workgroup)
  TileId id = PERSIST ? decode_tile_at<256, 256>(a, tcur, ntiles) : decode_tile<256, 256>(a);
  int m0 = id.m0, n0 = id.n0;
  const int nk = a.K / 64 / a.splitk;  // K-tiles of this block's K-slice

  uint32_t oSA[2][2], oSB[2][2];
  const uint32_t kbA = TA ? static_cast<uint32_t>(128 * a.lda) : 128u, kbB = TB ? static_cast<uint32_t>(128 * a.ldb) : 128u;
  const char* gA;
  const char* gB;
  // this lane's DMA sources and the uniform operand bases at the tile's first row /
  // column and first K-tile
  auto set_sources = [&]() {
    part_sources<TA>(oSA, a.lda, m0, a.M, wave, lane);
    part_sources<TB>(oSB, a.ldb, n0, a.N, wave, lane);
    const uint32_t kt0 = static_cast<uint32_t>(id.ks * nk);
    gA = static_cast<const char*>(a.A) + (TA ? m0 : m0 * a.lda) * 2 + kt0 * kbA;
    gB = static_cast<const char*>(a.B) + (TB ? n0 : n0 * a.ldb) * 2 + kt0 * kbB;
  };
  set_sources();

  // one part (P: 0 = A0, 1 = A1, 2 = B0, 3 = B1) of K-tile `tile` into its buffer,
  // or into the sink past the last tile (same wait accounting every phase)
  auto stage = [&](auto P, int tile) {
    constexpr int p = decltype(P)::value;
    const bool real = tile < nk;
    char* dst = lds + (real ? (tile & 1) * kBuf + p * kPart : kSink) + wave * 1024;
    // 32-bit tile offset (launch_ph8 requires each operand < 2 GiB): scalar math, no branches
    const char* g = (p < 2 ? gA : gB) + static_cast<uint32_t>(real ? tile : 0) * (p < 2 ? kbA : kbB);
    const uint32_t* o = p < 2 ? oSA[p & 1] : oSB[p & 1];
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(g + o[i]), (lds_void_t*)(dst + i * 8192), 16, 0, 0);
  };
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  using P2 = std::integral_constant<int, 2>;
  using P3 = std::integral_constant<int, 3>;

  int oA[TA ? 4 : 2], oB[2];
  part_offsets<TA, 4>(oA, wr * 64, lane);
  part_offsets<TB, 2>(oB, wc * 32, lane);

  f32x4 acc[8][4];

  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];
  auto rdA = [&](const char* part) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int f = 0; f < 4; ++f) fa[f][ks] = frag<TA>(part, oA, f, ks);
  };
  auto rdB = [&](const char* part, bf16x8 (&fb)[2][2]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int g = 0; g < 2; ++g) fb[g][ks] = frag<TB>(part, oB, g, ks);
  };
  // end of a phase's load segment: retire the part the next phase reads, meet the
  // partner group, then the quadrant's MFMAs at raised priority
  auto mid = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
  };
  auto end = [&]() {
    __builtin_amdgcn_s_setprio(0);
    barrier();
  };
  auto mma = [&](auto QM, auto QN, const bf16x8 (&fb)[2][2]) {
    constexpr int qm = decltype(QM)::value, qn = decltype(QN)::value;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g)
          acc[4 * qm + f][2 * qn + g] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[f][ks], fb[g][ks], acc[4 * qm + f][2 * qn + g], 0, 0, 0);
  };
  using Q0 = std::integral_constant<int, 0>;
  using Q1 = std::integral_constant<int, 1>;

  // prologue: B0, A0, B1, A1 of tile 0 and B0 of tile 1 (the order the loop's
  // phases -5 .. -1 would have staged them); vmcnt(6) retires B0 and A0 of tile 0
  auto prologue = [&]() {
    stage(P2{}, 0);
    stage(P0{}, 0);
    stage(P3{}, 0);
    stage(P1{}, 0);
    if constexpr (BAL) stage(P3{}, 1);
    else stage(P2{}, 1);
  };
  prologue();
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  barrier();
  for (;;) {  // one pass unless PERSIST
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (wave >= 4) barrier();  // stagger: waves 4-7 one barrier behind

  if constexpr (BAL) {
    // balanced reads (8, 4, 8, 4 per phase): a tile's two B quadrants alternate
    // between the register sets x / y, and phase 3 reads the NEXT tile's first B
    // part into the set phase 2 just released.  Tile v reads Bf(v) (B0 for even v,
    // B1 for odd) in phase 3 of tile v-1, A0 in 0, Bs(v) in 1, A1 in 2: every part
    // is staged 4 phases before its read and restaged 4 phases after it.
    bf16x8 fx[2][2], fy[2][2];
    rdB(lds + 2 * kPart, fx);  // Bf(0): retired by the prologue wait
    auto tile = [&](auto ODD, int u, bf16x8 (&bf)[2][2], bf16x8 (&bs)[2][2]) {
      constexpr bool odd = decltype(ODD)::value;
      // per-lane address state made opaque once per tile, so LICM cannot hoist every
      // phase's DMA and fragment address out of the loop into live registers
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(oSA[i >> 1][i & 1]), "+v"(oSB[i >> 1][i & 1]));
#pragma unroll
      for (int i = 0; i < (TA ? 4 : 2); ++i) asm volatile("" : "+v"(oA[i]));
      asm volatile("" : "+v"(oB[0]), "+v"(oB[1]));
      constexpr int pf = odd ? 3 : 2, ps = odd ? 2 : 3;  // this tile's Bf / Bs parts
      using QF = std::integral_constant<int, odd ? 1 : 0>;
      using QS = std::integral_constant<int, odd ? 0 : 1>;
      using PF = std::integral_constant<int, pf>;
      const char* buf = lds + (odd ? kBuf : 0);
      // phase 0: A0, quadrant (0, f)
      rdA(buf);
      stage(P0{}, u + 1);
      mid();
      mma(Q0{}, QF{}, bf);
      end();
      // phase 1: Bs, quadrant (0, s); DMA Bs(u+1) (= this tile's Bf part)
      rdB(buf + ps * kPart, bs);
      stage(PF{}, u + 1);
      mid();
      mma(Q0{}, QS{}, bs);
      end();
      // phase 2: A1, quadrant (1, s)
      rdA(buf + kPart);
      stage(P1{}, u + 1);
      mid();
      mma(Q1{}, QS{}, bs);
      end();
      // phase 3: Bf(u+1) into the released set, quadrant (1, f); DMA Bf(u+2)
      rdB(lds + (odd ? 0 : kBuf) + ps * kPart, bs);
      stage(PF{}, u + 2);
      mid();
      mma(Q1{}, QF{}, bf);
      end();
    };
    for (int u = 0; u < nk; u += 2) {  // nk even (launch_ph8)
      tile(std::false_type{}, u, fx, fy);
      tile(std::true_type{}, u + 1, fy, fx);
    }
  } else {
    for (int u = 0; u < nk; ++u) {
      const char* buf = lds + (u & 1) * kBuf;
      // phase 0: quadrant (0,0)
      rdB(buf + 2 * kPart, fb0);
      rdA(buf);
      stage(P0{}, u + 1);
      mid();
      mma(Q0{}, Q0{}, fb0);
      end();
      // phase 1: quadrant (0,1)
      rdB(buf + 3 * kPart, fb1);
      stage(P3{}, u + 1);
      mid();
      mma(Q0{}, Q1{}, fb1);
      end();
      // phase 2: quadrant (1,1)
      rdA(buf + kPart);
      stage(P1{}, u + 1);
      mid();
      mma(Q1{}, Q1{}, fb1);
      end();
      // phase 3: quadrant (1,0), fragments already in registers
      stage(P2{}, u + 2);
      mid();
      mma(Q1{}, Q0{}, fb0);
      end();
    }
  }
  if (wave < 4) barrier();  // end of the stagger: equal barrier counts
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  barrier();

  // PERSIST: the next tile's prologue parts go out now, under this tile's epilogue
  const int em0 = m0, en0 = n0;
  bool next = false;
  if constexpr (PERSIST) {
    tcur += gridDim.x;
    next = tcur < ntiles;
    if (next) {
      id = decode_tile_at<256, 256>(a, tcur, ntiles);
      m0 = id.m0;
      n0 = id.n0;
      set_sources();
      prologue();
    }
  }

  // epilogue: LDS-staged 16-byte rows, one pass per row quadrant (PERSIST: per fragment
  // row, in the LDS the prologue leaves free); the lane's 8 staged columns 8 (lane & 7)
  // .. +8 sit in column quadrant (lane & 7) >> 2
  float* ebuf = PERSIST ? reinterpret_cast<float*>(lds + kBuf) + wave * (16 * kEpiStride)
                        : reinterpret_cast<float*>(lds) + wave * kEpiWaveFloats;
  const int c8 = lane & 7;
  const int ncol = en0 + (c8 >> 2) * 128 + wc * 32 + 8 * (c8 & 3);
  auto store = [&](const DtpGemmArgs& e) {
    const uintptr_t cp = reinterpret_cast<uintptr_t>(e.C), ap = reinterpret_cast<uintptr_t>(e.aux);
    const bool vec = ncol + 8 <= e.N && e.ldc % 8 == 0 && (cp & 15) == 0 && (!e.aux || (e.ldaux % 8 == 0 && (ap & 15) == 0));
    float bias[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) bias[c] = (e.bias && ncol + c < e.N) ? e.bias[ncol + c] : 0.f;
    if constexpr (PERSIST) {
      static_for<0, 4>([&](auto IC) {
        constexpr int ii = decltype(IC)::value;
        fast_epilogue_pass<0, 0, 4, 16, ii>(e, acc, ebuf, bias, em0 + wr * 64 + 16 * ii, ncol, vec, lane);
      });
      static_for<0, 4>([&](auto IC) {
        constexpr int ii = decltype(IC)::value;
        fast_epilogue_pass<1, 0, 4, 16, ii>(e, acc, ebuf, bias, em0 + 128 + wr * 64 + 16 * ii, ncol, vec, lane);
      });
    } else {
      fast_epilogue_pass<0>(e, acc, ebuf, bias, em0 + wr * 64, ncol, vec, lane);
      fast_epilogue_pass<1>(e, acc, ebuf, bias, em0 + 128 + wr * 64, ncol, vec, lane);
    }
  };
  if constexpr (SPLIT) {  // raw f32 partial sums of this K-slice: work[ks][M][N]; splitk_reduce_kernel applies the epilogue
    DtpGemmArgs e = a;
    e.C = static_cast<char*>(a.work) + static_cast<long long>(id.ks) * a.M * a.N * 4;
    e.ldc = a.N;
    e.out_dtype = DTP_DT_F32;
    e.bias = nullptr;
    e.aux = nullptr;
    e.act = 0;
    e.accumulate = 0;
    e.alpha = 1.f;
    store(e);
  } else {
    store(a);
  }
  if (!next) break;
  // the next tile: its prologue parts (and this tile's stores) retired, every wave's
  // epilogue staging read before the K loop restages buffer 1
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  barrier();
  }  // for (;;)
}

// C = alpha * sum_s work[s] + bias (+ C): the epilogue of a split-K launch (f32 out,
// no activation).  Block = one output row x 1024 columns, 4 columns per thread (one
// 16-byte load per slice, contiguous per wave); the slices are read four at a time
// with all loads issued before any add.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(DtpGemmArgs a) {
  const int m = blockIdx.y, n = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (n >= a.N) return;
  const long long plane = static_cast<long long>(a.M) * a.N;
  const float* w = static_cast<const float*>(a.work) + static_cast<long long>(m) * a.N + n;
  float* c = static_cast<float*>(a.C) + static_cast<long long>(m) * a.ldc + n;
  const bool vec = n + 4 <= a.N && a.N % 4 == 0 && a.ldc % 4 == 0 && (reinterpret_cast<uintptr_t>(a.C) & 15) == 0;
  if (vec) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    int s = 0;
    for (; s + 4 <= a.splitk; s += 4) {
      f32x4 x[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) x[q] = *reinterpret_cast<const f32x4*>(w + (s + q) * plane);
#pragma unroll
      for (int q = 0; q < 4; ++q) v += x[q];
    }
    for (; s < a.splitk; ++s) v += *reinterpret_cast<const f32x4*>(w + s * plane);  // splitk = 2
    f32x4* cv = reinterpret_cast<f32x4*>(c);
    f32x4 o = {0.f, 0.f, 0.f, 0.f}, b = o;
    if (a.accumulate) o = *cv;
    if (a.bias) b = f32x4{a.bias[n], a.bias[n + 1], a.bias[n + 2], a.bias[n + 3]};
    *cv = o + (a.alpha * v + b);  // the order of the unsplit epilogue: C + (alpha acc + bias)
  } else {
    for (int q = 0; q < 4 && n + q < a.N; ++q) {
      float x = 0.f;
      for (int s = 0; s < a.splitk; ++s) x += w[s * plane + q];
      c[q] = (a.accumulate ? c[q] : 0.f) + (a.alpha * x + (a.bias ? a.bias[n + q] : 0.f));
    }
  }
}

}  // namespace ph8

// variant 0: balanced reads, 2: reads 12/4/8/0 per phase; -1: by layout (dtp_gemm's
// default).  (Variant 1, the two wave groups in lockstep instead of staggered, measured
// 8-20 % slower on every layout, profiles/gemm_r3_ph8, and was removed.)
template <bool BAL, bool SPLIT>
static void launch_lay(const DtpGemmArgs& a, hipStream_t s, dim3 g, dim3 b) {
  switch ((a.trans_a ? 2 : 0) | (a.trans_b ? 1 : 0)) {
    case 0: hipLaunchKernelGGL((ph8::gemm_ph8_kernel<false, false, BAL, SPLIT>), g, b, 0, s, a); break;
    case 1: hipLaunchKernelGGL((ph8::gemm_ph8_kernel<false, true, BAL, SPLIT>), g, b, 0, s, a); break;
    case 2: hipLaunchKernelGGL((ph8::gemm_ph8_kernel<true, false, BAL, SPLIT>), g, b, 0, s, a); break;
    default: hipLaunchKernelGGL((ph8::gemm_ph8_kernel<true, true, BAL, SPLIT>), g, b, 0, s, a); break;
  }
}

// Split-K plan for problems with too few 256x256 tiles to fill the chip -- the weight
// gradient dW = dz^T h of a 1024-2048-wide layer has 16-64 tiles and K = batch: s
// K-slices per tile, s a power of two with tiles * s <= 256 (one workgroup per CU)
// and every slice an even number (>= 8) of K-tiles; the slices' f32 partial sums go
// to the caller's workspace and splitk_reduce_kernel applies the epilogue.  An f32
// output without activation epilogues only; 0 = no plan.
int ph8_split_plan(const DtpGemmArgs& a) {
  if (a.out_dtype != DTP_DT_F32 || a.act || a.aux || a.K % 64) return 0;
  const long long tiles = (long long)((a.M + 255) / 256) * ((a.N + 255) / 256);
  if (tiles >= 128) return 0;
  const int nk = a.K / 64;
  int s = 1;
  while (tiles * s * 2 <= 256 && nk % (s * 4) == 0 && nk / (s * 2) >= 8) s *= 2;
  return s > 1 ? s : 0;
}

long long ph8_split_bytes(const DtpGemmArgs& a, int splitk) { return 4LL * splitk * a.M * a.N; }

int launch_ph8(const DtpGemmArgs& a, hipStream_t s, int variant) {
  const long long tiles = (long long)((a.M + 255) / 256) * ((a.N + 255) / 256) * a.splitk;
  const dim3 g((unsigned)tiles), b(ph8::kThreads);
  // default (-1): the balanced reads (profiles/gemm_r3_ph8)
  if (variant < 0) variant = 0;
  if ((a.K / 64 / a.splitk) % 2) variant = 2;  // the balanced schedule runs K-tiles in pairs
  if (variant == 3 && a.splitk == 1) {  // persistent balanced walk: one workgroup per CU (a multiple of 8)
    int cus = 256, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    const long long grid = tiles < cus ? (tiles + 7) / 8 * 8 : cus / 8 * 8;
    const dim3 gp((unsigned)(grid > 0 ? grid : 8));
    switch ((a.trans_a ? 2 : 0) | (a.trans_b ? 1 : 0)) {
      case 0: hipLaunchKernelGGL((ph8::gemm_ph8_kernel<false, false, true, false, true>), gp, b, 0, s, a); break;
      case 1: hipLaunchKernelGGL((ph8::gemm_ph8_kernel<false, true, true, false, true>), gp, b, 0, s, a); break;
      case 2: hipLaunchKernelGGL((ph8::gemm_ph8_kernel<true, false, true, false, true>), gp, b, 0, s, a); break;
      default: hipLaunchKernelGGL((ph8::gemm_ph8_kernel<true, true, true, false, true>), gp, b, 0, s, a); break;
    }
    return check_launch("dtp_gemm(8-phase LDS-DMA 256x256, persistent)");
  }
  if (variant == 3) variant = 0;
  if (a.splitk > 1) variant == 2 ? launch_lay<false, true>(a, s, g, b) : launch_lay<true, true>(a, s, g, b);
  else variant == 2 ? launch_lay<false, false>(a, s, g, b) : launch_lay<true, false>(a, s, g, b);
  if (a.splitk > 1) {
    int e = check_launch("dtp_gemm(8-phase LDS-DMA 256x256, split-K)");
    if (e) return e;
    hipLaunchKernelGGL(ph8::splitk_reduce_kernel, dim3((a.N + 1023) / 1024, a.M), dim3(256), 0, s, a);
    return check_launch("dtp_gemm(split-K reduction)");
  }
  return check_launch("dtp_gemm(8-phase LDS-DMA 256x256)");
}

}  // namespace gemm
}  // namespace dtp
