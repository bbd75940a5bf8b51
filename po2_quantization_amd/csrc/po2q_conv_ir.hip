// A whole MobileNetV2 inverted-residual block in ONE launch (reference models/mobilenet.py:53-134;
// MobileViT's MV2Block has the same shape, models/mobile_vit.py:131-239): three QuantizedConv2d
// forwards (quantized_conv.py:32-38) with their eval BatchNorms and activations,
//     h = act1(bn1(conv1x1(x, Q(We))))          expand (absent when the expand ratio is 1: h = x)
//     d = act2(bn2(dwconv3x3(h, Q(Wd), stride, pad 1)))
//     y = act3(bn3(conv1x1(d, Q(Wp))) (+ x))    project; the identity shortcut when stride 1, Cin == Cout
// The hidden activations h and d never leave the CU.
//
// Why: at CIFAR size every layer of MobileNetV2 is a few MB of activations and a few microseconds
// of work, so the layer-by-layer forward is ~50 latency-bound launches whose HBM traffic is
// dominated by the 6x-wide hidden tensors (written by the expand, read + written by the depthwise,
// read by the project).  Here a block owns a band of R output rows of G images (G > 1 only when
// one image is one band) and walks the hidden channels in chunks of CHK = 32 KC:
//   prologue   the band's input rows (+ the depthwise halo) of x -> LDS fp32 [pixel][Cin + pad];
//   per chunk  expand: each wave owns one pair of 16-channel tiles and walks the 16-pixel groups on
//              v_mfma_f32_16x16x32_bf16 (A = the exact hi / mid / lo bf16 split of x, B = the expand
//              layer's pointwise pack), bn1 + act1 -> hidden fp32 [channel][pixel];  barrier;
//              depthwise 3x3: fp32 FMAs in conv_dw3's tap order (the quantized depthwise weight
//              is exact fp32), bn2 + act2, exact split -> bf16 planes [output pixel][CHK];
//              barrier;
//              project: every wave accumulates its (output-pixel group, output-channel tile) units
//              over the chunk's KC k-steps (B = the project layer's pointwise pack);
//   epilogue   bn3 (+ the residual x) + act3 -> y.
// Latency, not arithmetic, bounds a block at these sizes (a few hundred MFMAs per chunk), so no
// weight load sits on the critical path: each wave's expand and project B fragments for the next
// chunk are loaded into registers right after it used this chunk's (they land under the other
// phases), and the chunk's depthwise weights + BN vectors are loaded before the expand and parked
// in LDS after it.
// Weights come from the three layers' own packs (qconv2d_pack_batch: the pointwise [ks][nt][lane]
// bf16 fragments + scale multiplier, the depthwise plain quantized fp32 copy), so every weight is
// still quantized in every forward.  Arithmetic per layer is the layer kernels' own (conv_pw's
// MFMA order and epilogue expression, conv_dw3's fma order and epilogue), so the block equals
// the layer chain up to the pointwise kernels' k-split summation order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#ifdef PO2Q_IR_STAMPS
#include <cstdio>
#include <vector>
#endif

#include "po2q_epi.h"
#include "po2q_internal.h"
#include "po2q_rows_dev.h"
#include "po2q_x3_dev.h"

namespace po2q {

namespace {
constexpr int kIrThreads = 512;  // 8 waves
constexpr int kIrWaves = kIrThreads / 64;
constexpr int kIrKse = 5;     // expand k-steps held in registers: Cin <= 160
constexpr int kIrBatch = 8;   // independent global loads per thread in the staging loops
constexpr int kIrCw = 12;     // staged depthwise parameters per hidden channel: 9 taps, bn scale, shift, pad
constexpr size_t kIrLds = 150 * 1024;
// project units one wave holds B fragments for, by k-steps per chunk (<= 8 fragments = 32 VGPRs:
// the prefetched fragments are live through the depthwise phase, whose tap reads need the room)
constexpr int ir_umax(int kc) { return kc >= 8 ? 1 : (kc >= 4 ? 2 : (kc >= 2 ? 4 : 8)); }
}  // namespace

struct IrArgs {
    int N, Cin, H, W, Ch, Cout, S, Ho, Wo;
    int G, R, RI, nbands;  // images per block, output / input rows per band, bands per image
    int KSe, NTe, KSp, NTp;  // expand / project k-steps (32 ch) and 16-channel output tiles
    int xs;                // x row stride in LDS (floats): 32 KSe + 4
    int P, PG, Po, HP;     // input pixels, their 16-groups, output pixels (x16) of a block; hidden row stride
    const uint4* we;       // expand pack (NULL: h = x)
    const float* we_scale;
    const float* wd;  // depthwise quantized weight [Ch][9]
    const uint4* wp;  // project pack
    const float* wp_scale;
    const float *ps1, *pb1, *ps2, *pb2, *ps3, *pb3;
    int act1, act2, act3;
    const float* res;      // residual [N, Cout, Ho, Wo] or NULL
    int off_hid, off_dpl, off_cw;  // LDS byte offsets
    unsigned* stamps;  // PO2Q_IR_STAMPS diagnostic builds only: per (block, wave) phase cycle sums
};

// Diagnostic build (-DPO2Q_IR_STAMPS, `make irstamps`): s_memtime phase stamps, never in the
// product build.  Phases: 0 prologue, 1 barrier A, 2 expand, 3 expand prefetch issue, 4 depthwise
// parameters to LDS (their load wait), 5 barrier B, 6 depthwise, 7 barrier C, 8 project,
// 9 project prefetch issue, 10 epilogue.
[[maybe_unused]] constexpr int kIrPhases = 11;
#ifdef PO2Q_IR_STAMPS
#define IRS(i)                                                                           \
    do {                                                                                 \
        __builtin_amdgcn_sched_barrier(0);                                               \
        unsigned long long t_;                                                           \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");        \
        __builtin_amdgcn_sched_barrier(0);                                               \
        ph_[i] += (unsigned)(t_ - tprev_);                                               \
        tprev_ = t_;                                                                     \
    } while (0)
#else
#define IRS(i) \
    do {       \
    } while (0)
#endif

// Block barrier over LDS only: every LDS access of this wave retired, then s_barrier.  Not
// __syncthreads: its release fence also waits for every global load in flight (vmcnt(0)), which would
// serialise the register prefetches of the next chunk's weights with this chunk's phases.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS: x [16 PG][xs] fp32 (expand only) | hidden chunk [CHK][HP] fp32 | d planes 3 x [Po][CHK] bf16 |
// the chunk's depthwise parameters [CHK][12] fp32.  KC: project k-steps per chunk (CHK = 32 KC).
template <int KC>
__global__ __launch_bounds__(kIrThreads) void conv_ir(const float* __restrict__ x, float* __restrict__ y, IrArgs a) {
    constexpr int CHK = 32 * KC;
    constexpr int UMAX = ir_umax(KC);
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
#ifdef PO2Q_IR_STAMPS
    unsigned ph_[kIrPhases] = {};
    unsigned long long tprev_;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tprev_)::"memory");
#endif
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, pl = lane & 15;
    const int band = blockIdx.x % a.nbands, n0 = (blockIdx.x / a.nbands) * a.G;
    const int oy0 = band * a.R, Rb = min(a.R, a.Ho - oy0);
    const int iy0 = max(0, oy0 * a.S - 1), iy1 = min(a.H - 1, (oy0 + Rb - 1) * a.S + 1);
    const int IMG = a.RI * a.W, IMGo = a.R * a.Wo;  // LDS pixels of one image (input / output)
    const bool expand = a.we != nullptr;
    float* xl = reinterpret_cast<float*>(lds);
    float* hid = reinterpret_cast<float*>(lds + a.off_hid);
    unsigned char* dpl = lds + a.off_dpl;
    float* cw = reinterpret_cast<float*>(lds + a.off_cw);
    constexpr int drow = CHK * 2;     // bytes per output pixel of a d plane
    const int dplane = a.Po * drow;   // bytes per d plane
    const int nunits = a.Po / 16 * a.NTp;
    constexpr uint4 z4 = {0u, 0u, 0u, 0u};

    // ---- register-held B fragments: this wave's expand tile pair and its project units
    const int tp = wave % KC;  // the expand tile pair this wave owns in every chunk
    uint4 bwe[kIrKse][2];
    float e1s[2], e1b[2];
    auto load_bwe = [&](int c0n) __attribute__((always_inline)) {
        const int ntile = min(CHK, a.Ch - c0n) / 16;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const bool tok = 2 * tp + t < ntile;  // wave-uniform
            const int tile = c0n / 16 + 2 * tp + t;
#pragma unroll
            for (int ks = 0; ks < kIrKse; ++ks)
                bwe[ks][t] = (tok && ks < a.KSe) ? a.we[((int64_t)ks * a.NTe + tile) * 64 + lane] : z4;
            const int h = 16 * tile + pl;
            e1s[t] = (tok && a.ps1) ? a.ps1[h] : 1.0f;
            e1b[t] = (tok && a.pb1) ? a.pb1[h] : 0.0f;
        }
    };
    uint4 bwp[UMAX][KC];
    auto load_bwp = [&](int c0n) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < UMAX; ++i) {
            const int u = wave + kIrWaves * i;
            const int ot = u % a.NTp;
#pragma unroll
            for (int k2 = 0; k2 < KC; ++k2) {
                const int ks = c0n / 32 + k2;
                bwp[i][k2] = (u < nunits && ks < a.KSp) ? a.wp[((int64_t)ks * a.NTp + ot) * 64 + lane] : z4;
            }
        }
    };
    if (expand) load_bwe(0);
    load_bwp(0);

    // the band's input pixel px (image, row iy0 + ry, column) of channel c; 0 outside
    auto x_at = [&](int c, int px) -> float {
        const int img = px / IMG, r = px - img * IMG;
        const int ry = r / a.W, ix = r - ry * a.W;
        const int iy = iy0 + ry;
        if (img >= a.G || n0 + img >= a.N || iy > iy1 || c >= a.Cin) return 0.0f;
        return x[(((int64_t)(n0 + img) * a.Cin + c) * a.H + iy) * a.W + ix];
    };
    // global -> LDS staging, kIrBatch independent loads in flight per thread (a loop of one load
    // and one LDS store per iteration pays a full memory latency per element)
    auto stage = [&](int total, auto&& src, auto&& dst) __attribute__((always_inline)) {
        for (int base = tid; base < total; base += kIrThreads * kIrBatch) {
            float v[kIrBatch];
#pragma unroll
            for (int j = 0; j < kIrBatch; ++j) {
                const int u = base + kIrThreads * j;
                v[j] = u < total ? src(u) : 0.0f;
            }
#pragma unroll
            for (int j = 0; j < kIrBatch; ++j) {
                const int u = base + kIrThreads * j;
                if (u < total) dst(u, v[j]);
            }
        }
    };
    if (expand) {
        const int cinp = 32 * a.KSe, P16 = 16 * a.PG;
        stage(
            P16 * cinp, [&](int u) { return x_at(u / P16, u - (u / P16) * P16); },
            [&](int u, float v) { xl[(u - (u / P16) * P16) * a.xs + u / P16] = v; });
    }
    const float se = expand ? *a.we_scale : 1.0f;
    const float sp = *a.wp_scale;

    floatx4 acc[UMAX];
#pragma unroll
    for (int i = 0; i < UMAX; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};

    constexpr int CWPT = (CHK * 11 + kIrThreads - 1) / kIrThreads;  // staged parameters per thread
    for (int c0 = 0; c0 < a.Ch; c0 += CHK) {
        const int CH = min(CHK, a.Ch - c0);  // a multiple of 16
        // the chunk's depthwise taps and BN vectors: loaded now, parked in LDS after the expand
        float cwv[CWPT];
#pragma unroll
        for (int j = 0; j < CWPT; ++j) {
            const int idx = tid + kIrThreads * j;
            const int hc = idx / 11, k = idx - hc * 11;
            float v = 0.0f;
            if (hc < CH) {
                const int h = c0 + hc;
                v = k < 9 ? a.wd[h * 9 + k] : (k == 9 ? (a.ps2 ? a.ps2[h] : 1.0f) : (a.pb2 ? a.pb2[h] : 0.0f));
            }
            cwv[j] = v;
        }
        IRS(0);
        lds_barrier();  // x staged / the previous chunk's depthwise reads of hid and cw retired
        IRS(1);
        // ---- expand (or copy x) -> hid [CH][HP] fp32
        if (expand) {
            const int ntile = CH / 16, t0 = 2 * tp, nt = min(2, ntile - t0);
            if (nt > 0) {  // wave-uniform
                for (int pg = wave / KC; pg < a.PG; pg += kIrWaves / KC) {
                    floatx4 c[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
                    const float* xr = xl + (16 * pg + pl) * a.xs + 8 * g;
#pragma unroll
                    for (int ks = 0; ks < kIrKse; ++ks) {
                        if (ks >= a.KSe) break;
                        const floatx4 v0 = *reinterpret_cast<const floatx4*>(xr + 32 * ks);
                        const floatx4 v1 = *reinterpret_cast<const floatx4*>(xr + 32 * ks + 4);
                        const uint32_t b[8] = {__float_as_uint(v0[0]), __float_as_uint(v0[1]),
                                               __float_as_uint(v0[2]), __float_as_uint(v0[3]),
                                               __float_as_uint(v1[0]), __float_as_uint(v1[1]),
                                               __float_as_uint(v1[2]), __float_as_uint(v1[3])};
                        uint4 hi, mid, lo;
                        split3(b, hi, mid, lo);
                        const bf16x8 ah = __builtin_bit_cast(bf16x8, hi), am = __builtin_bit_cast(bf16x8, mid),
                                     al = __builtin_bit_cast(bf16x8, lo);
#pragma unroll
                        for (int t = 0; t < 2; ++t) {
                            if (t < nt) {  // wave-uniform
                                const bf16x8 bw = __builtin_bit_cast(bf16x8, bwe[ks][t]);
                                c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bw, c[t], 0, 0, 0);
                                c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bw, c[t], 0, 0, 0);
                                c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bw, c[t], 0, 0, 0);
                            }
                        }
                    }
                    // lane: hidden channel c0 + 16 (t0 + t) + pl, pixels 16 pg + 4 g .. + 3 (conv_pw's epilogue)
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        if (t >= nt) break;
                        const int hc = 16 * (t0 + t) + pl;
                        floatx4 v;
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            float q = c[t][e] * se + 0.0f;
                            q = q * e1s[t] + e1b[t];
                            v[e] = epi_act(q, a.act1);
                        }
                        *reinterpret_cast<floatx4*>(hid + hc * a.HP + 16 * pg + 4 * g) = v;
                    }
                }
            }
            IRS(2);
            if (c0 + CHK < a.Ch) load_bwe(c0 + CHK);  // the next chunk's: lands under this chunk's other phases
            IRS(3);
        } else {
            stage(
                CH * a.P, [&](int u) { return x_at(c0 + u / a.P, u - (u / a.P) * a.P); },
                [&](int u, float v) { hid[(u / a.P) * a.HP + u - (u / a.P) * a.P] = v; });
        }
#pragma unroll
        for (int j = 0; j < CWPT; ++j) {
            const int idx = tid + kIrThreads * j;
            if (idx < CHK * 11) {
                const int hc = idx / 11, k = idx - hc * 11;
                cw[hc * kIrCw + k] = cwv[j];
            }
        }
        IRS(4);
        lds_barrier();
        IRS(5);
        // ---- depthwise 3x3 (pad 1, stride S), bn2 + act2, split -> d planes [Po][CHK]
        // branch-free: the 9 tap offsets of the output pixel (clamped into the band, a select zeroes
        // the padding taps) are shared by its 8 channels, so every LDS read is unconditional and
        // the 72 of a unit are independent
        for (int u = tid; u < a.Po * (CHK / 8); u += kIrThreads) {
            const int oc = u / a.Po, op = u - oc * a.Po;
            const int img = op / IMGo, r = op - img * IMGo;
            const int ry = r / a.Wo, ox = r - ry * a.Wo;
            const int oy = oy0 + min(ry, Rb - 1);
            const bool ok = img < a.G && ry < Rb;
            int toff[9];
            bool tin[9];
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
                const int iy = oy * a.S - 1 + rr;
                const int iyc = min(max(iy, iy0), iy1);
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    const int ix = ox * a.S - 1 + t;
                    toff[rr * 3 + t] = min(img, a.G - 1) * IMG + (iyc - iy0) * a.W + min(max(ix, 0), a.W - 1);
                    tin[rr * 3 + t] = iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
                }
            }
            uint32_t b[8];
            // two channels per batch: their 18 tap reads and 6 parameter reads are all issued
            // before the first FMA (one LDS round trip per batch, not one per tap)
#pragma unroll
            for (int e0 = 0; e0 < 8; e0 += 2) {
                float hv[2][9];
                floatx4 wv[2][3];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int hc = 8 * oc + e0 + e;
                    const float* hp = hid + hc * a.HP;
#pragma unroll
                    for (int k = 0; k < 9; ++k) hv[e][k] = hp[toff[k]];
#pragma unroll
                    for (int j = 0; j < 3; ++j) wv[e][j] = *reinterpret_cast<const floatx4*>(cw + hc * kIrCw + 4 * j);
                }
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int hc = 8 * oc + e0 + e;
                    float s = 0.0f;
#pragma unroll
                    for (int k = 0; k < 9; ++k) s = fmaf(tin[k] ? hv[e][k] : 0.0f, wv[e][k >> 2][k & 3], s);
                    float q = s + 0.0f;  // conv_dw3's epilogue (no bias)
                    q = q * wv[e][2][1] + wv[e][2][2];
                    const float v = epi_act(q, a.act2);
                    b[e0 + e] = (ok && hc < CH) ? __float_as_uint(v) : 0u;
                }
            }
            uint4 hi, mid, lo;
            split3(b, hi, mid, lo);
            const int off = op * drow + 16 * oc;
            *reinterpret_cast<uint4*>(dpl + off) = hi;
            *reinterpret_cast<uint4*>(dpl + dplane + off) = mid;
            *reinterpret_cast<uint4*>(dpl + 2 * dplane + off) = lo;
        }
        IRS(6);
        lds_barrier();
        IRS(7);
        // ---- project: the chunk's k-steps into this wave's units
        const int nks = (CH + 31) / 32;
#pragma unroll
        for (int i = 0; i < UMAX; ++i) {
            const int u = wave + kIrWaves * i;
            if (u >= nunits) break;
            const int opg = u / a.NTp;
#pragma unroll
            for (int k2 = 0; k2 < KC; ++k2) {
                if (k2 >= nks) break;
                const bf16x8 bw = __builtin_bit_cast(bf16x8, bwp[i][k2]);
                const int off = (16 * opg + pl) * drow + 16 * (4 * k2 + g);
#pragma unroll
                for (int p3 = 0; p3 < 3; ++p3) {
                    const bf16x8 af =
                        __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(dpl + p3 * dplane + off));
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw, acc[i], 0, 0, 0);
                }
            }
        }
        IRS(8);
        if (c0 + CHK < a.Ch) load_bwp(c0 + CHK);
        IRS(9);
    }

    // ---- epilogue (conv_pw's): lane holds output channel 16 ot + pl, output pixels 16 opg + 4 g .. + 3.
    // Two passes: every residual and BN load of the wave first, then the stores (one round trip).
    // Indices fit 32 bits (ir_plan: N Cout H W < 2^31).
    int yi[UMAX][4];
    float rv[UMAX][4], s3[UMAX], b3[UMAX];
#pragma unroll
    for (int i = 0; i < UMAX; ++i) {
        const int u = wave + kIrWaves * i;
        const int opg = u / a.NTp, ot = u - opg * a.NTp;
        const int k = 16 * ot + pl;
        const bool kok = u < nunits && k < a.Cout;
        s3[i] = (kok && a.ps3) ? a.ps3[k] : 1.0f;
        b3[i] = (kok && a.pb3) ? a.pb3[k] : 0.0f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int op = 16 * opg + 4 * g + e;
            const int img = op / IMGo, r = op - img * IMGo;
            const int ry = r / a.Wo, ox = r - ry * a.Wo;
            const bool ok = kok && img < a.G && n0 + img < a.N && ry < Rb;
            yi[i][e] = ok ? (((n0 + img) * a.Cout + k) * a.Ho + oy0 + ry) * a.Wo + ox : -1;
            rv[i][e] = (ok && a.res) ? a.res[yi[i][e]] : 0.0f;
        }
    }
#pragma unroll
    for (int i = 0; i < UMAX; ++i) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float v = acc[i][e] * sp + 0.0f;
            v = v * s3[i] + b3[i];
            if (a.res) v += rv[i][e];
            if (yi[i][e] >= 0) y[yi[i][e]] = epi_act(v, a.act3);
        }
    }
#ifdef PO2Q_IR_STAMPS
    IRS(10);
    if (lane == 0 && a.stamps)
        for (int i = 0; i < kIrPhases; ++i) a.stamps[((size_t)blockIdx.x * kIrWaves + wave) * kIrPhases + i] = ph_[i];
#endif
}

// ------------------------------------------------------------------ small images --
// conv_ir_small: the block for images of at most 16 pixels (MobileNetV2 @32 from its 4x4 stage on:
// 13 of 17 blocks).  There the chunked kernel above runs ~15 chunks of a few dozen MFMAs, each
// behind three block barriers, and its 16-row pixel tiles hold 1-4 real pixels.  Here a block owns
// G images whose G H W <= 16 pixels fill ONE 16-row MFMA tile, and the hidden channels are split
// over the waves in 32-channel slices that each wave runs end to end with no block barrier:
//   expand (A = the block's pre-split x planes, B = the slice's two expand tiles) -> bn1 + act1 ->
//   the wave's own LDS [32 ch][16 px] -> depthwise 3x3 (lane = channel, 8 output pixels) -> bn2 +
//   act2 -> exact split -> the wave's own bf16 planes [16 px][32 ch] -> project: one k-step into
//   the wave's NTW output tiles (partial sums over its slices, in registers).
// The next slice's B fragments and depthwise parameters are loaded right after their phase used
// the current ones.  At the end the partial sums of the waves meet in LDS and are added in a fixed
// wave order (deterministic), then bn3 (+ the residual) + act3 and the store.  With more than NTW
// output tiles the waves form TG groups, each over its own tiles (the expand / depthwise work of a
// slice is then repeated per group: it is the small part at these sizes).
constexpr int kIrsWave = 5120;  // per-wave LDS: hidden [32][16] fp32 (2 KiB) + 3 bf16 planes [16][32] (3 KiB)

template <int NTW>
__global__ __launch_bounds__(kIrThreads) void conv_ir_small(const float* __restrict__ x, float* __restrict__ y,
                                                            IrArgs a, int TG) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, pl = lane & 15;
    const int n0 = blockIdx.x * a.G;
    const int HW = a.H * a.W, HWo = a.Ho * a.Wo;
    const int P = a.G * HW, Po = a.G * HWo;  // <= 16 each
    const int cinp = 32 * a.KSe;
    const int xplane = 16 * cinp * 2;
    unsigned char* xpl = lds;
    float* hidw = reinterpret_cast<float*>(lds + 3 * xplane + wave * kIrsWave);
    unsigned char* dplw = lds + 3 * xplane + wave * kIrsWave + 2048;
    constexpr uint4 z4 = {0u, 0u, 0u, 0u};

    // ---- x -> exact split planes [16 px][cinp] (pixels past P and channels past Cin: zero)
    for (int u = tid; u < 16 * (cinp / 8); u += kIrThreads) {
        const int px = u / (cinp / 8), oc = u - px * (cinp / 8);
        const int img = px / HW, p = px - img * HW;
        const bool ok = px < P && n0 + img < a.N;
        uint32_t b[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int c = 8 * oc + e;
            b[e] = (ok && c < a.Cin) ? __float_as_uint(x[((int64_t)(n0 + img) * a.Cin + c) * HW + p]) : 0u;
        }
        uint4 hi, mid, lo;
        split3(b, hi, mid, lo);
        const int off = px * cinp * 2 + 16 * oc;
        *reinterpret_cast<uint4*>(xpl + off) = hi;
        *reinterpret_cast<uint4*>(xpl + xplane + off) = mid;
        *reinterpret_cast<uint4*>(xpl + 2 * xplane + off) = lo;
    }
    const float se = *a.we_scale, sp = *a.wp_scale;
    const int tg = wave % TG, sw = wave / TG, nsw = kIrWaves / TG;
    const int nslices = a.Ch / 32;

    // ---- register-held operands of a slice
    uint4 bwe[kIrKse][2];
    float e1s[2], e1b[2];
    auto load_e = [&](int sl) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int tile = 2 * sl + t;
#pragma unroll
            for (int ks = 0; ks < kIrKse; ++ks)
                bwe[ks][t] = ks < a.KSe ? a.we[((int64_t)ks * a.NTe + tile) * 64 + lane] : z4;
            e1s[t] = a.ps1 ? a.ps1[16 * tile + pl] : 1.0f;
            e1b[t] = a.pb1 ? a.pb1[16 * tile + pl] : 0.0f;
        }
    };
    float dwv[11];  // the depthwise taps, bn2 scale and shift of this lane's channel
    const int dc = lane & 31, dh = lane >> 5;
    auto load_d = [&](int sl) __attribute__((always_inline)) {
        const int h = 32 * sl + dc;
#pragma unroll
        for (int k = 0; k < 9; ++k) dwv[k] = a.wd[h * 9 + k];
        dwv[9] = a.ps2 ? a.ps2[h] : 1.0f;
        dwv[10] = a.pb2 ? a.pb2[h] : 0.0f;
    };
    uint4 bwp[NTW];
    auto load_p = [&](int sl) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NTW; ++i) {
            const int ot = tg * NTW + i;
            bwp[i] = ot < a.NTp ? a.wp[((int64_t)sl * a.NTp + ot) * 64 + lane] : z4;
        }
    };
    floatx4 acc[NTW];
#pragma unroll
    for (int i = 0; i < NTW; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (sw < nslices) {
        load_e(sw);
        load_d(sw);
        load_p(sw);
    }
    lds_barrier();  // x planes

    for (int sl = sw; sl < nslices; sl += nsw) {
        const bool more = sl + nsw < nslices;
        // ---- expand: this slice's two hidden tiles
        floatx4 c[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int ks = 0; ks < kIrKse; ++ks) {
            if (ks >= a.KSe) break;
            const int off = pl * cinp * 2 + 16 * (4 * ks + g);
            const bf16x8 ah = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(xpl + off));
            const bf16x8 am = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(xpl + xplane + off));
            const bf16x8 al = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(xpl + 2 * xplane + off));
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const bf16x8 bw = __builtin_bit_cast(bf16x8, bwe[ks][t]);
                c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bw, c[t], 0, 0, 0);
                c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bw, c[t], 0, 0, 0);
                c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bw, c[t], 0, 0, 0);
            }
        }
        // lane: hidden channel 16 t + pl of the slice, pixels 4 g .. 4 g + 3 (conv_pw's epilogue)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            floatx4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float q = c[t][e] * se + 0.0f;
                q = q * e1s[t] + e1b[t];
                v[e] = epi_act(q, a.act1);
            }
            *reinterpret_cast<floatx4*>(hidw + (16 * t + pl) * 16 + 4 * g) = v;
        }
        if (more) load_e(sl + nsw);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own hidden writes
        // ---- depthwise: lane = channel dc of the slice, output pixels dh, dh + 2, .. (<= 16)
#pragma unroll 2
        for (int k8 = 0; k8 < 8; ++k8) {
            const int op = dh + 2 * k8;
            const int img = op / HWo, r = op - img * HWo;
            const int oy = r / a.Wo, ox = r - oy * a.Wo;
            const bool ok = op < Po && n0 + img < a.N;
            const int imc = min(img, a.G - 1);
            float hv[9];
            bool tin[9];
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
                const int iy = oy * a.S - 1 + rr;
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    const int ix = ox * a.S - 1 + t;
                    tin[rr * 3 + t] = iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
                    const int pix = imc * HW + min(max(iy, 0), a.H - 1) * a.W + min(max(ix, 0), a.W - 1);
                    hv[rr * 3 + t] = hidw[dc * 16 + pix];
                }
            }
            float s = 0.0f;
#pragma unroll
            for (int k = 0; k < 9; ++k) s = fmaf(tin[k] ? hv[k] : 0.0f, dwv[k], s);
            float q = s + 0.0f;  // conv_dw3's epilogue
            q = q * dwv[9] + dwv[10];
            const float v = ok ? epi_act(q, a.act2) : 0.0f;
            uint16_t h16, m16, l16;
            split1(__float_as_uint(v), h16, m16, l16);
            const int off = op * 64 + dc * 2;
            *reinterpret_cast<uint16_t*>(dplw + off) = h16;
            *reinterpret_cast<uint16_t*>(dplw + 1024 + off) = m16;
            *reinterpret_cast<uint16_t*>(dplw + 2048 + off) = l16;
        }
        if (more) load_d(sl + nsw);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own d-plane writes
        // ---- project: the slice's k-step into this wave's output tiles
        {
            const int off = pl * 64 + 16 * g;
            const bf16x8 ah = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(dplw + off));
            const bf16x8 am = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(dplw + 1024 + off));
            const bf16x8 al = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(dplw + 2048 + off));
#pragma unroll
            for (int i = 0; i < NTW; ++i) {
                if (tg * NTW + i >= a.NTp) break;  // wave-uniform
                const bf16x8 bw = __builtin_bit_cast(bf16x8, bwp[i]);
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bw, acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bw, acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bw, acc[i], 0, 0, 0);
            }
        }
        if (more) load_p(sl + nsw);
    }

    // ---- the waves' partial sums meet in LDS (aliasing the planes: every wave is past them)
    lds_barrier();
    floatx4* red = reinterpret_cast<floatx4*>(lds);
#pragma unroll
    for (int i = 0; i < NTW; ++i) red[(wave * NTW + i) * 64 + lane] = acc[i];
    lds_barrier();
    // output tile ft (group ft / NTW, local tile ft % NTW): the sum over that group's waves in wave
    // order; lane: output channel 16 ft + pl, pixels 4 g .. 4 g + 3
    for (int ft = wave; ft < a.NTp; ft += kIrWaves) {
        const int grp = ft / NTW, i = ft - grp * NTW;
        floatx4 v = red[(grp * NTW + i) * 64 + lane];
        for (int w = grp + TG; w < kIrWaves; w += TG) v += red[(w * NTW + i) * 64 + lane];
        const int k = 16 * ft + pl;
        if (k >= a.Cout) continue;
        const float s3 = a.ps3 ? a.ps3[k] : 1.0f, b3 = a.pb3 ? a.pb3[k] : 0.0f;
        int yi[4];
        float rv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int op = 4 * g + e;
            const int img = op / HWo, r = op - img * HWo;
            const bool ok = op < Po && n0 + img < a.N;
            yi[e] = ok ? ((n0 + img) * a.Cout + k) * HWo + r : -1;
            rv[e] = (ok && a.res) ? a.res[yi[e]] : 0.0f;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float q = v[e] * sp + 0.0f;
            q = q * s3 + b3;
            if (a.res) q += rv[e];
            if (yi[e] >= 0) y[yi[e]] = epi_act(q, a.act3);
        }
    }
}

// ------------------------------------------------------------------ planning --
namespace {

bool ir_geom(IrPlan& q, int64_t Cin, int64_t H, int64_t W, int64_t Cout, int64_t S, bool expand, int64_t R,
             int64_t G, int KC) {
    const int64_t Ho = (H - 1) / S + 1, Wo = (W - 1) / S + 1;
    const int64_t RI = std::min<int64_t>(H, (R - 1) * S + 3);
    const int64_t P = G * RI * W, PG = (P + 15) / 16, Po = (G * R * Wo + 15) / 16 * 16;
    const int64_t xs = 32 * ((Cin + 31) / 32) + 4;
    const int64_t HP = 16 * PG + 4;  // 16-byte shift between channel rows: conflict-free float4 stores
    const int64_t CHK = 32 * KC;
    const size_t xb = expand ? (size_t)16 * PG * xs * 4 : 0;
    const size_t hb = (size_t)CHK * HP * 4;
    const size_t db = (size_t)3 * Po * CHK * 2;
    const size_t cb = (size_t)CHK * kIrCw * 4;
    if (xb + hb + db + cb > kIrLds) return false;
    const int64_t units = Po / 16 * ((Cout + 15) / 16);
    if (units > (int64_t)kIrWaves * ir_umax(KC)) return false;
    q.G = (int)G; q.R = (int)R; q.RI = (int)RI; q.nbands = (int)((Ho + R - 1) / R); q.CHK = (int)CHK;
    q.P = (int)P; q.PG = (int)PG; q.Po = (int)Po; q.HP = (int)HP; q.xs = (int)xs;
    q.lds = xb + hb + db + cb; q.off_hid = xb; q.off_dpl = xb + hb; q.off_cw = xb + hb + db;
    return true;
}

}  // namespace

// Geometry: whole images when one fits (G > 1 of them while a block has < 64 output pixels and
// the grid keeps >= 512 blocks), else the tallest band of one image that fits the LDS budget and
// the project unit cap; then the widest chunk (KC = 8, 4, 2, 1 k-steps, no wider than the hidden
// width) whose B fragments the waves can hold and whose buffers fit: small images get few, wide
// chunks (fewer barriers).
bool ir_plan(IrPlan& ip, int64_t N, int64_t Cin, int64_t H, int64_t W, int64_t Ch, int64_t Cout, int64_t S,
             bool expand) {
    if (N <= 0 || Cin <= 0 || H <= 0 || W <= 0 || Ch <= 0 || Cout <= 0 || (S != 1 && S != 2)) return false;
    if (Ch % 16 != 0 || (!expand && Ch != Cin) || Ch > 4096 || Cout > 1024) return false;
    if (expand && Cin > 32 * kIrKse) return false;  // the expand B fragments live in registers
    if (!expand && Cin > 4096) return false;
    if (N * Cin * H * W >= INT32_MAX || N * Cout * H * W >= INT32_MAX || N * Ch * H * W >= ((int64_t)1 << 40))
        return false;
    const int64_t Ho = (H - 1) / S + 1, Wo = (W - 1) / S + 1;
    const int64_t NTp = (Cout + 15) / 16;
    // small images: the slice-per-wave kernel (PO2Q_IR_SMALL=0: off, A/B)
    const char* sm = getenv("PO2Q_IR_SMALL");
    // Default only for images of 9..16 pixels (one image per block): 18 vs 25 us per block at 4x4 bs 256,
    // where at 2x2 / 1x1 (several images per block, each block streaming all the weights) it loses to
    // the layer launches (profiles/r04_ir_small_ab.jsonl); PO2Q_IR_SMALL=1 takes every size <= 16.
    const bool small_all = sm && sm[0] == '1';
    if (expand && H * W <= 16 && (H * W >= 9 || small_all) && Ch % 32 == 0 && Cin <= 32 * kIrKse && NTp <= 24 &&
        !(sm && sm[0] == '0')) {
        IrPlan q{};
        int64_t G = 1;
        while (G * 2 * H * W <= 16 && G * 2 <= N) G *= 2;  // one 16-pixel tile of G images
        q.small = 1;
        q.tg = NTp <= 12 ? 1 : 2;
        const int64_t per = (NTp + q.tg - 1) / q.tg;
        q.ntw = per <= 4 ? 4 : (per <= 8 ? 8 : 12);
        q.G = (int)G;
        q.R = (int)Ho;
        q.RI = (int)H;
        q.nbands = 1;
        q.CHK = 32;
        q.P = (int)(G * H * W);
        q.Po = 16;
        const size_t xb = (size_t)3 * 16 * (32 * ((Cin + 31) / 32)) * 2;
        q.lds = std::max(xb + (size_t)kIrWaves * kIrsWave, (size_t)kIrWaves * q.ntw * 1024);
        q.blocks = (N + G - 1) / G;
        ip = q;
        return true;
    }
    // The chunked kernel for larger images is opt-in (PO2Q_IR_LARGE=1): at the sizes measured it
    // ties or loses to the three layer launches replayed from a HIP graph (profiles/r04_ir_ab.jsonl),
    // so by default those blocks run as the layers (po2q_qconv2d_ir_supported says 0).
    {
        const char* lg = getenv("PO2Q_IR_LARGE");
        if (!(lg && lg[0] == '1')) return false;
    }
    IrPlan q{};
    bool found = false;
    int64_t R = Ho, G = 1;
    for (; R >= 1 && !found; --R) found = ir_geom(q, Cin, H, W, Cout, S, expand, R, 1, 1);
    if (!found) return false;
    R = q.R;
    // PO2Q_IR_MINBLOCKS (A/B knob): the fewest blocks image grouping may leave (default 512)
    int64_t minblocks = 512;
    if (const char* e = getenv("PO2Q_IR_MINBLOCKS")) minblocks = std::max(1, atoi(e));
    if (R == Ho) {
        while (G * Ho * Wo < 64 && N / (G * 2) >= minblocks) {
            IrPlan q2{};
            if (!ir_geom(q2, Cin, H, W, Cout, S, expand, R, G * 2, 1)) break;
            q = q2;
            G *= 2;
        }
    }
    // the widest chunk that fits (q holds the KC = 1 geometry, which does)
    const int64_t ksteps = (Ch + 31) / 32;
    for (int KC = 8; KC > 1; KC /= 2)
        if (KC <= ksteps && ir_geom(q, Cin, H, W, Cout, S, expand, R, G, KC)) break;
    ip = q;
    ip.blocks = (N + G - 1) / G * q.nbands;
    return true;
}

hipError_t launch_conv_ir(const IrPlan& ip, const float* x, float* y, int N, int Cin, int H, int W, int Ch, int Cout,
                          int S, const uint16_t* we, const float* we_scale, const float* wd, const uint16_t* wp,
                          const float* wp_scale, const IrEpi& e, hipStream_t s) {
    IrArgs a;
    a.N = N; a.Cin = Cin; a.H = H; a.W = W; a.Ch = Ch; a.Cout = Cout; a.S = S;
    a.Ho = (H - 1) / S + 1; a.Wo = (W - 1) / S + 1;
    a.G = ip.G; a.R = ip.R; a.RI = ip.RI; a.nbands = ip.nbands;
    a.KSe = (Cin + 31) / 32; a.NTe = (Ch + 15) / 16; a.KSp = (Ch + 31) / 32; a.NTp = (Cout + 15) / 16;
    a.xs = ip.xs; a.P = ip.P; a.PG = ip.PG; a.Po = ip.Po; a.HP = ip.HP;
    a.we = reinterpret_cast<const uint4*>(we);
    a.we_scale = we_scale;
    a.wd = wd;
    a.wp = reinterpret_cast<const uint4*>(wp);
    a.wp_scale = wp_scale;
    a.ps1 = e.ps1; a.pb1 = e.pb1; a.ps2 = e.ps2; a.pb2 = e.pb2; a.ps3 = e.ps3; a.pb3 = e.pb3;
    a.act1 = e.act1; a.act2 = e.act2; a.act3 = e.act3;
    a.res = e.res;
    a.off_hid = (int)ip.off_hid;
    a.off_dpl = (int)ip.off_dpl;
    a.off_cw = (int)ip.off_cw;
    a.stamps = nullptr;
    auto go = [&](auto kern) -> hipError_t {
        if (ip.lds > 64 * 1024) {
            const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)kIrLds);
            if (attr != hipSuccess) return attr;
        }
#ifdef PO2Q_IR_STAMPS
        const size_t nst = (size_t)ip.blocks * kIrWaves * kIrPhases;
        if (getenv("PO2Q_STAMPS") && hipMalloc(&a.stamps, nst * 4) == hipSuccess) {
            (void)hipMemsetAsync(a.stamps, 0, nst * 4, s);
            hipLaunchKernelGGL(kern, dim3((unsigned)ip.blocks), dim3(kIrThreads), ip.lds, s, x, y, a);
            std::vector<unsigned> h(nst);
            (void)hipStreamSynchronize(s);
            (void)hipMemcpy(h.data(), a.stamps, nst * 4, hipMemcpyDeviceToHost);
            (void)hipFree(a.stamps);
            fprintf(stderr, "[po2q ir stamps] N=%d Cin=%d H=%d Ch=%d Cout=%d S=%d CHK=%d G=%d blocks=%lld, cycles/block by wave:\n",
                    N, Cin, H, Ch, Cout, S, ip.CHK, ip.G, (long long)ip.blocks);
            for (int w = 0; w < kIrWaves; ++w) {
                double tot = 0;
                fprintf(stderr, "  wave %d:", w);
                for (int i = 0; i < kIrPhases; ++i) {
                    double sum = 0;
                    for (int64_t b = 0; b < ip.blocks; ++b) sum += h[((size_t)b * kIrWaves + w) * kIrPhases + i];
                    sum /= (double)ip.blocks;
                    tot += sum;
                    fprintf(stderr, " %d:%.0f", i, sum);
                }
                fprintf(stderr, " total %.0f\n", tot);
            }
            return hipGetLastError();
        }
#endif
        hipLaunchKernelGGL(kern, dim3((unsigned)ip.blocks), dim3(kIrThreads), ip.lds, s, x, y, a);
        return hipGetLastError();
    };
    if (ip.small) {
        auto gs = [&](auto kern) -> hipError_t {
            if (ip.lds > 64 * 1024) {
                const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)kIrLds);
                if (attr != hipSuccess) return attr;
            }
            hipLaunchKernelGGL(kern, dim3((unsigned)ip.blocks), dim3(kIrThreads), ip.lds, s, x, y, a, ip.tg);
            return hipGetLastError();
        };
        switch (ip.ntw) {
            case 4: return gs(conv_ir_small<4>);
            case 8: return gs(conv_ir_small<8>);
            case 12: return gs(conv_ir_small<12>);
            default: return hipErrorInvalidValue;
        }
    }
    switch (ip.CHK) {
        case 32: return go(conv_ir<1>);
        case 64: return go(conv_ir<2>);
        case 128: return go(conv_ir<4>);
        case 256: return go(conv_ir<8>);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace po2q
