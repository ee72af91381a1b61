// On-device PPO update (SB3 2.x PPO.train) for small minibatches, one workgroup-resident launch.
//
// Reference: PPO('MlpPolicy', env, n_steps=10, learning_rate=1e-3, ent_coef=0.01) with SB3
// defaults (/root/reference/vectorized_env.py:126-131): n_epochs passes over the rollout buffer in
// shuffled minibatches of batch_size = 64; per minibatch the clipped surrogate + vf_coef * value
// loss + ent_coef * entropy loss, backward, clip_grad_norm_(0.5), Adam(eps 1e-5).  The torch
// restatement of the same update is ppo.py (graph / eager paths); this kernel is its fused form.
//
// Why one workgroup per network: a minibatch step depends on the previous step's parameters,
// and a 64-sample step of this 9,669-parameter MLP is ~1.8 MFLOP -- far too little to spread
// over the chip, and ~100 tiny launches per step in torch (~430 us replayed as a HIP graph).
// The actor and the critic only couple through the global gradient norm, so by default they run
// as two workgroups on two CUs (FENV_PPO_SPLIT below); FENV_PPO_SPLIT=0 is the one-workgroup
// form of the same code.  Here the parameters,
// their gradients and the minibatch's activations live in LDS (152 KB), each thread keeps the
// Adam moments of the ~19 parameters it owns in registers, and the loop runs every minibatch of
// every epoch inside one launch.  The 64-deep contractions run on the MFMA pipe: layer 2, W2
// gradients and dL/dh1 (the three 32 x 32 x 64 tiles per wave) in split-f16 form -- x = hi + lo,
// hi = x's leading 11 bits, lo = the remainder rounded to f16, three v_mfma_f32_32x32x16_f16
// (hi*lo, lo*hi, hi*hi) per 16-deep chunk, exact products and fp32 accumulation, the dropped
// lo*lo and lo's rounding < 2^-21 relative; dL/dz2 scaled by a power of two into f16's range
// first, exactly undone -- and layer 1, the heads and W1 gradients on fp32
// v_mfma_f32_16x16x4f32; the parameter and gradient images are padded (lx) so the operand reads
// are bank-conflict free.  tanh is
// 1 - 2 / (1 + e^2x) on v_exp/v_rcp and the gradient norm is summed by the threads that write
// the gradient entries.  Results match the torch path to summation-order rounding plus the
// tanh's < 3e-7 (tests/test_gpu_rollout.py).
//
// Work split per minibatch (B <= 64 samples, 8 waves, 2 per SIMD); every contraction runs over
// all 64 sample rows (rows >= B hold finite stale values and are multiplied by zeroed dL/dz):
//   forward  layer 1: one 16-unit x 64-sample block per wave (16x16x4 MFMA, K = 8);
//            layer 2: one 32 x 32 tile (net, sample rows, hidden cols) per wave, 32 MFMAs;
//            heads mu / value: one 16-sample tile per wave (16x16x4, K = 64) -> per-sample slots.
//   loss     wave 0, lane = sample: log-prob, ratio, clipped surrogate, value loss, and the
//            per-sample gradients w.r.t. mu, value, log_std (torch's min/clamp subgradients).
//   backward head weight grads (16x16x4 tile of hidden rows per wave) and dL/dz2 in place of the
//            same wave's H2 columns (rows >= B zeroed); one 32 x 32 tile of both W2 grads and
//            dL/dh1 per wave, dL/dz1 in place of layer 1 after a barrier; W1 grads (16x16x4).
//   update   global grad 2-norm (per-thread sums of the entries each wrote, block reduction), clip,
//            Adam with bias correction.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <set>
#include <type_traits>
#include <utility>

#include "fenv.h"
#include "fenv_internal.h"
#include "policy_device.h"

namespace fenvk {

constexpr int kPB = 64;                         // max samples per minibatch
constexpr int kPT = 512;                        // threads (8 waves; 256-VGPR budget)
constexpr int kNW = kPT / 64;                   // waves
static_assert(kNW == 8, "the MFMA tile-to-wave maps below assume 8 waves");
constexpr int kRow = kHid + 1;                  // padded activation row
constexpr int kMaxP = 9680;                     // >= policy_param_count(8) = 9,669
constexpr int kPerT = (kMaxP + kPT - 1) / kPT;  // parameters owned per thread (Adam moments)
constexpr int kMaxPL = kMaxP + kMaxP / 64 + 1;  // padded LDS image of kMaxP parameters

// Parameter p lives at LDS float lx(p): one pad float after every 64.  Every 64 x 64 hidden
// weight block starts at a multiple of 64 (PLayout: the blocks before it are 64 (D + 1) floats),
// so its rows land at stride 65 = kRow and MFMA operand reads down a column or along a row hit
// 64 distinct banks.
__device__ __forceinline__ int lx(int p) { return p + (p >> 6); }

// LDS layout (floats)
constexpr int oPW = 0;                        // [kMaxPL] parameters (padded image, lx)
constexpr int oPG = oPW + kMaxPL;             // [kMaxPL] gradients (same image)
constexpr int oPO = oPG + kMaxPL;             // [kPB][9] observations (zero-padded to 8)
constexpr int oPH1 = oPO + kPB * 9;           // [2][kPB][kRow] layer-1 tanh, then dL/dz1
constexpr int oPH2 = oPH1 + 2 * kPB * kRow;   // [2][kPB][kRow] layer-2 tanh, then dL/dz2
constexpr int oPS = oPH2 + 2 * kPB * kRow;    // [16][kPB] per-sample scalars
constexpr int oPR = oPS + 16 * kPB;           // [64] reduction scratch
constexpr int oPB1 = oPR + 64;                // [2][64] b1-gradient partial sums (split launch)
constexpr int kPPOLds = oPB1 + 2 * kHid;
constexpr size_t kPPOLdsBytes = (size_t)kPPOLds * sizeof(float);
static_assert(kPPOLdsBytes <= 160 * 1024, "fused PPO update exceeds the 160 KiB LDS of a CU");
static_assert(2 * (kHid * 9 + kHid * (kHid + 1)) + 3 * (kHid + 1) + 2 <= kMaxP,
              "parameter image too small for D = 8");

// per-sample scalar slots
enum { sA0 = 0, sA1, sOLP, sADV, sRET, sGMU0, sGMU1, sGV, sMU0, sMU1, sVAL,
       sPL, sCF, sGL0, sGL1, sVLS };  // the last five: per-sample loss terms (split launch)
constexpr int kEnt = 56;              // R slot: the entropy (split launch)
constexpr int kZM = 40;               // R slots [kZM, kZM + 8): per-wave max |dL/dz2| (wave w)

struct PPOArgs {
    float *params, *exp_avg, *exp_avg_sq, *step;
    const float *obs, *act, *old_log_prob, *adv, *ret;
    const int64_t *perm;
    int64_t n;
    int32_t D, n_epochs, batch_size;
    ppo_hparams hp;
    double *stats;
    uint64_t *xch;  // split launch: the two blocks' {minibatch + 1, partial grad norm^2} words
                    // (the caller's workspace: one set per PPO instance, not per device)
    // gradient mode (ppo_grad, data-parallel update): one minibatch of this rank's rows, loss
    // means over the GLOBAL minibatch of b_global samples, advantages normalised with the global
    // minibatch's mean / std; the gradient goes to grad[P] instead of clip + Adam
    float *grad;
    float inv_bg, adv_mean, adv_std;
    int32_t adv_norm_on, ent_once;
    // test hook (fenv_test_ppo_inject): the critic block never posts its partial and the actor's
    // wait budget is short, so the launch ends as a lost exchange does
    int32_t inject_lost;
    // Adam's moment rates as torch uses them: fp32 of (1 - beta) formed in double from the
    // Python float beta (torch/optim/adam.py: lerp_(grad, 1 - beta1), addcmul_(.., value=1 -
    // beta2)), not 1 - fp32(beta): for beta2 = 0.999 the two differ by 1.3e-5 relative, a
    // coherent bias of every second moment (adam_rates below)
    float omb1, omb2;
};

// fp32 of (1 - b) for the double b whose shortest decimal form rounds to the fp32 beta (0.9,
// 0.999: what a Python float beta becomes in ppo_hparams), as torch computes the rate in double.
static float adam_rate(float beta) {
    char buf[32];
    double d = (double)beta;
    for (int prec = 1; prec <= 9; ++prec) {
        snprintf(buf, sizeof buf, "%.*g", prec, (double)beta);
        if (strtof(buf, nullptr) == beta) {
            d = strtod(buf, nullptr);
            break;
        }
    }
    return (float)(1.0 - d);
}
static void adam_rates(const ppo_hparams &hp, float &omb1, float &omb2) {
    omb1 = adam_rate(hp.beta1);
    omb2 = adam_rate(hp.beta2);
}

// Split launch (FENV_PPO_SPLIT): the actor and the critic each on their own CU.  The two networks'
// forward, loss and backward are independent; the only coupling is clip_grad_norm_'s global norm,
// exchanged once per minibatch through two 64-bit words in L2 (the working blocks are 0 and 8,
// which the dispatcher places on the same XCD).  Each block runs the unsplit kernel's four waves
// of its network on one CU, one wave per SIMD, and updates only its own parameters.
#ifndef FENV_PPO_SPLIT
#define FENV_PPO_SPLIT 1
#endif
constexpr int kPTS = 256;   // threads per block, split launch
constexpr int kPerTS = 20;  // parameters owned per thread, split launch (actor: 4,868 at D = 8)

// tanh x = 1 - 2 / (1 + e^(2x)) on v_exp_f32 + v_rcp_f32 (absolute error < 3e-7 over the whole
// range, +-1 at +-inf) instead of the ~30-instruction libm tanhf: the update's forward only has
// to match torch's tanh to fp32 rounding noise (tests/test_gpu_rollout.py bounds the update)
__device__ __forceinline__ float tanh_u(float x) {
    const float e = __builtin_amdgcn_exp2f(x * 2.88539008177792681f);  // 2 log2(e)
    return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + e);
}

// two at a time: the same operations as float2, so the multiply / add /
// fma steps issue as packed fp32
// (An accurate small-argument tanh -- an odd polynomial below |x| = 0.55, where the exp form
// loses up to 1.4e-3 relative, 1.6e-7 absolute -- costs 0.5 us per minibatch and lands no closer to
// torch at the reference config, measured in rounds 3 and 4: profiles/ab/r3_ppo_tanh_ab.txt,
// profiles/ab/r4_ppo_precision_ab.txt; source at commit 2c54623.)
__device__ __forceinline__ void tanh_u2(float x0, float x1, float &y0, float &y1) {
    using f2 = float __attribute__((ext_vector_type(2)));
    const f2 x = {x0, x1};
    const f2 t = x * 2.88539008177792681f;  // 2 log2(e)
    const f2 e = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
    const f2 d = 1.0f + e;
    const f2 r = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    const f2 y = 1.0f - 2.0f * r;
    y0 = y.x;
    y1 = y.y;
}

#ifndef FENV_PPO_UDZ
#define FENV_PPO_UDZ 4  // unroll of the dL/dz2 loop (16 steps)
#endif
// Column sum of an activation-gradient image (rows at stride kRow): the bias gradient.  Rows
// b >= B of dL/dz2 and dL/dz1 are exact zeros, so summing all kPB rows adds only zeros.
__device__ __forceinline__ float col_sum(const float *z, int B) {
    (void)B;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
    for (int b = 0; b < kPB; b += 4) {
        a0 += z[b * kRow];
        a1 += z[(b + 1) * kRow];
        a2 += z[(b + 2) * kRow];
        a3 += z[(b + 3) * kRow];
    }
    return (a0 + a1) + (a2 + a3);
}

// Sum over the 64 lanes, in every lane: DPP row shifts and row
// broadcasts (a fixed order; six VALU ops and one v_readlane) instead of six dependent
// ds_bpermute round trips of the xor butterfly.
__device__ __forceinline__ float wsum(float v) {
    int x = __float_as_int(v);
    x = __float_as_int(__int_as_float(x) + __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false)));
    x = __float_as_int(__int_as_float(x) + __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false)));
    x = __float_as_int(__int_as_float(x) + __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xe, false)));
    x = __float_as_int(__int_as_float(x) + __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xc, false)));
    x = __float_as_int(__int_as_float(x) + __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false)));
    x = __float_as_int(__int_as_float(x) + __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false)));
    return __int_as_float(__builtin_amdgcn_readlane(x, 63));
}

// Max over the 64 lanes of non-negative values (same DPP pattern as wsum: lanes shifted in
// from outside a row read 0, the identity here), wave-uniform.
__device__ __forceinline__ float wmax_nn(float v) {
    int x = __float_as_int(v);
    x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false))));
    x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false))));
    x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xe, false))));
    x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xc, false))));
    x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false))));
    x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false))));
    return __int_as_float(__builtin_amdgcn_readlane(x, 63));
}

#ifndef FENV_PPO_DUMP_GRAD
#define FENV_PPO_DUMP_GRAD 0
#endif
#ifndef FENV_PPO_PROFILE
#define FENV_PPO_PROFILE 0  // 1 / 2: per-phase shader-clock totals of the actor / critic block -> stats[4..15] (diagnostic build)
#endif
#if FENV_PPO_PROFILE
#define FENV_PPO_PHASE(i)                                            \
    if (tid == 0) {                                                  \
        const uint64_t now = __builtin_readcyclecounter();           \
        prof[i] += (double)(now - tlast);                            \
        tlast = now;                                                 \
    }
#else
#define FENV_PPO_PHASE(i)
#endif

template <bool SPLIT, bool GRAD = false>
__global__ __launch_bounds__(SPLIT ? kPTS : kPT) void k_ppo_update(PPOArgs g) {
    static_assert(!GRAD || SPLIT, "gradient mode is built on the split (two-CU) layout");
    constexpr int NT = SPLIT ? kPTS : kPT;     // threads of a working block
    constexpr int KP = SPLIT ? kPerTS : kPerT;  // Adam slots per thread
    if (SPLIT && (blockIdx.x & 7) != 0) return;  // split: blocks 0 and 8 work (one XCD)
    const int net_b = SPLIT ? (int)(blockIdx.x >> 3) : 0;  // split: this block's network
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float *W = sm + oPW, *G = sm + oPG, *O = sm + oPO, *H1 = sm + oPH1, *H2 = sm + oPH2;
    float *S = sm + oPS, *R = sm + oPR, *B1P = sm + oPB1;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wl = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave of this block
    const int w = wl + (SPLIT ? 4 * net_b : 0);               // wave index of the unsplit kernel
    const int D = g.D;
    const PLayout L(D);
    const int P = L.total;
    const ppo_hparams hp = g.hp;
    const float ar1 = g.omb1, ar2 = g.omb2;  // Adam's (1 - beta) rates (PPOArgs)
    // parameter of Adam slot q of this thread (P: none).  Split: the block's network only --
    // actor = pi* layers, action head, log_std; critic = vf* layers, value head.
    auto own = [&](int q) -> int {
        int i = tid + q * NT;
        if (!SPLIT) return i < P ? i : P;
        if (net_b == 0) {
            const int n0 = L.vf0W - L.pi0W, n1 = L.valW - L.actW;
            if (i < n0) return L.pi0W + i;
            i -= n0;
            if (i < n1) return L.actW + i;
            i -= n1;
            return i < 2 ? L.logstd + i : P;
        }
        const int n0 = L.actW - L.vf0W, n1 = L.logstd - L.valW;
        if (i < n0) return L.vf0W + i;
        i -= n0;
        return i < n1 ? L.valW + i : P;
    };

    for (int p = tid; p < P; p += NT) W[lx(p)] = g.params[p];
    // activations and observations start finite: the MFMA contractions run over all 64 rows
    // and a partial minibatch's unused rows (multiplied by zeros) must not hold NaN bit patterns
    for (int q = tid; q < 4 * kPB * kRow; q += NT) H1[q] = 0.0f;  // H1 and H2 are contiguous
    for (int q = tid; q < kPB * 9; q += NT) O[q] = 0.0f;
    float m[KP], v[KP];  // Adam moments of the parameters this thread owns
#pragma unroll
    for (int q = 0; q < KP; ++q) {
        const int p = own(q);
        m[q] = (!GRAD && p < P) ? g.exp_avg[p] : 0.0f;
        v[q] = (!GRAD && p < P) ? g.exp_avg_sq[p] : 0.0f;
    }
    float step = GRAD ? 0.0f : g.step[0];
    // beta^step for the bias corrections, carried in double and multiplied by beta per minibatch
    // (one double pow per launch): (float) of it is the correctly rounded fp32 power torch's
    // _foreach_pow gives -- exp2f(step * log2f(beta)) was up to 1 ulp off, up to 6e-5 relative in
    // 1 - beta2^step at the first steps -- and a double pow per minibatch costs ~1.2 us
    double pw1 = 1.0, pw2 = 1.0;
    if (!GRAD) {
        pw1 = pow((double)hp.beta1, (double)step);
        pw2 = pow((double)hp.beta2, (double)step);
    }
    // split: the LDS index of each Adam slot's parameter, fixed for the launch; a slot without a
    // parameter points at the pad float after parameter 63 (lx leaves one after every 64; no
    // read ever uses it), so the Adam loop runs branch-free
    constexpr int kPadIx = 64;
    int lp[SPLIT ? KP : 1];
    if constexpr (SPLIT) {
#pragma unroll
        for (int q = 0; q < KP; ++q) {
            const int p = own(q);
            lp[q] = p < P ? lx(p) : kPadIx;
        }
    }
    bool partner_lost = false;  // split launch: the other block's norm exchange timed out
    double st_pl = 0.0, st_vl = 0.0, st_el = 0.0, st_cf = 0.0;
#if FENV_PPO_PROFILE
    double prof[11] = {};
    uint64_t tlast = __builtin_readcyclecounter();
#endif
    __syncthreads();

    const int64_t n = g.n;
    const int bs = g.batch_size;
    // Gather pipeline (a thread moves OPT observation values -- B * 8 <= OPT * NT -- and, for
    // tid < B, one sample's act / old_log_prob / adv / ret).  The minibatch's values were loaded
    // into registers during the previous minibatch, from perm indices loaded one minibatch
    // before that, so no gather waits on a dependent global load (the loop's barriers wait on
    // LDS only).  Minibatch k = (epoch, start) in the loop's order; kMB = minibatches per epoch.
    const int64_t kMB = (n + bs - 1) / bs;
    const int64_t nmb = kMB * (int64_t)g.n_epochs;
    constexpr int OPT = (kPB * 8 + NT - 1) / NT;
    // minibatch positions (epoch, start) advance incrementally (no 64-bit division per minibatch)
    auto advance = [&](int64_t &e, int64_t &sk) {
        sk += bs;
        if (sk >= n) {
            sk = 0;
            ++e;
        }
    };
    auto perm_rows = [&](int64_t e, int64_t s0k, int64_t (&ro)[OPT], int64_t &rs) {  // rows this thread gathers
        rs = -1;
#pragma unroll
        for (int j = 0; j < OPT; ++j) ro[j] = -1;
        if (e >= g.n_epochs) return;
        const int Bk = (int)((n - s0k) < bs ? (n - s0k) : bs);
        const int64_t *pp = g.perm + e * n + s0k;
#pragma unroll
        for (int j = 0; j < OPT; ++j)
            if (tid + j * NT < Bk * 8) ro[j] = pp[(tid + j * NT) >> 3];
        if (tid < Bk) rs = pp[tid];
    };
    auto load_rows = [&](const int64_t (&ro)[OPT], int64_t rs, float (&po)[OPT], float (&ps)[5]) {
        const int i = tid & 7;  // NT is a multiple of 8: every slot j of a thread has column i
#pragma unroll
        for (int j = 0; j < OPT; ++j) po[j] = (ro[j] >= 0 && i < D) ? g.obs[ro[j] * D + i] : 0.0f;
        if (rs >= 0) {
            ps[0] = g.act[2 * rs];
            ps[1] = g.act[2 * rs + 1];
            ps[2] = g.old_log_prob[rs];
            ps[3] = g.adv[rs];
            ps[4] = g.ret[rs];
        }
    };
    float po[OPT], ps[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    int64_t ro_n[OPT], rs_n;  // perm rows of the next minibatch
    {
        int64_t ro0[OPT], rs0;
        perm_rows(0, 0, ro0, rs0);
        load_rows(ro0, rs0, po, ps);
        int64_t e1 = 0, s1 = 0;
        advance(e1, s1);
        perm_rows(e1, s1, ro_n, rs_n);
    }
    // Advantage normalisation of a Bk-sample minibatch (whole wave; lane l < Bk holds sample
    // l's advantage a).  It depends on the data only, so the split launch's actor block does it
    // one minibatch ahead, while its norm exchange waits on L2 (adv_nx: wave 0's lanes).
    auto adv_norm = [&](int Bk, float a) -> float {
        if constexpr (GRAD)  // the global minibatch's statistics, computed by the caller
            return g.adv_norm_on ? (a - g.adv_mean) / (g.adv_std + 1e-8f) : a;
        if (!(hp.normalize_advantage && Bk > 1)) return a;
        const float invBk = 1.0f / (float)Bk;
        const float x = lane < Bk ? a : 0.0f;
        const float mean = wsum(x) * invBk;
        const float d = lane < Bk ? x - mean : 0.0f;
        const float sd = __builtin_sqrtf(wsum(d * d) / (float)(Bk - 1));
        return (x - mean) / (sd + 1e-8f);
    };
    int64_t e2 = 0, s2 = 0;  // position of minibatch kmb + 2
    advance(e2, s2);
    advance(e2, s2);
    // Late gather (split launch): the next minibatch's observations and
    // per-sample inputs go to LDS at the END of a minibatch, after its last O / S read and
    // while thread 0 waits on the norm exchange, instead of at the start of the next one.
    constexpr bool kLate = SPLIT && !GRAD;
    auto gather_store = [&](int Bk, float adv_val) {
#pragma unroll
        for (int j = 0; j < OPT; ++j) {
            const int e = tid + j * NT;
            if (e < Bk * 8) O[(e >> 3) * 9 + (e & 7)] = po[j];
        }
        if (tid < Bk) {
            S[sA0 * kPB + tid] = ps[0];
            S[sA1 * kPB + tid] = ps[1];
            S[sOLP * kPB + tid] = ps[2];
            S[sADV * kPB + tid] = adv_val;
            S[sRET * kPB + tid] = ps[4];
        }
    };
    float adv_nx = 0.0f;
    if (SPLIT && net_b == 0 && wl == 0) adv_nx = adv_norm((int)(n < bs ? n : bs), ps[3]);
    // Adam split (split launch): a minibatch's Adam step updates the slots
    // holding layer 1 (W1, b1: slots 0..kKA-1 of every thread, PLayout puts them first) before
    // the barrier, and the other slots (W2, b2, heads, log_std) only in the next minibatch's
    // layer-1 phase, whose MFMAs and tanh never read them: the scheduler fills layer 1's
    // latencies with the register-only Adam arithmetic.  Same operations, same results.
    constexpr bool kAS = SPLIT && !GRAD;
    constexpr bool kPK = SPLIT && KP % 2 == 0;
    // ceil((64 D + 64) / 256) <= 3 for D <= 8 (4 when packed: slot pairs)
    constexpr int kKA = kAS ? (kPK ? 4 : 3) : KP;
    // dL/dz1 in the other network's H1 half (split launch: each block owns
    // the whole LDS image but runs one network, so that half is free)
    constexpr bool kZ1S = SPLIT && !FENV_PPO_DUMP_GRAD;
    // split launch: the loss wave writes per-sample terms; waves 1-3 take the sums afterwards
    constexpr bool kSpread = SPLIT;
    const int stat_tid = kSpread ? 64 : 0;  // the thread accumulating the loss statistics
    constexpr bool kB2 = SPLIT;  // split: the b2 gradient summed by the head-gradient phase's lanes
    constexpr bool kB1 = SPLIT;  // split: b1-gradient partial sums from the dL/dz1 writers
    constexpr bool kAcc2 = SPLIT;  // split: 16-step 16x16x4 MFMA chains as two interleaved accumulators
    constexpr bool kDZP = SPLIT;
    constexpr bool kBCW = SPLIT && !GRAD;
    constexpr int kBC = 60;  // R slots: this minibatch's Adam step size and 1 / sqrt(bc2)
    const int zb = kZ1S ? (net_b ^ 1) : 0;  // H1 half holding dL/dz1 (unsplit: per network)
    // Adam with the clip coefficient (fused form)
    float a_coef = 0.f, a_ss = 0.f, a_ib = 0.f;  // clip coef, step size, 1/sqrt(bc2)
    float gq[SPLIT ? KP : 1], wq[SPLIT ? KP : 1];
    auto adam_slot = [&](int q) {
        const int p = SPLIT ? 0 : own(q);  // split: every slot (spare ones hit the pad)
        if (p < P) {
            const int ix = SPLIT ? lp[q] : lx(p);
            const float gr = (SPLIT ? gq[q] : G[ix]) * a_coef;
            m[q] = __builtin_fmaf(ar1, gr - m[q], m[q]);
            v[q] = __builtin_fmaf(ar2, gr * gr, v[q] * hp.beta2);
            const float den = __builtin_fmaf(__builtin_amdgcn_sqrtf(v[q]), a_ib, hp.eps);
            const float wn = __builtin_fmaf(-a_ss, m[q] * __builtin_amdgcn_rcpf(den),
                                            SPLIT ? wq[q] : W[ix]);
            W[ix] = wn;
        }
    };
    // Split launch: two slots per step as float2 arithmetic, so the compiler
    // issues packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two lanes' worth of fp32
    // per VALU slot); same operations and roundings as two adam_slot calls (fused form)
    using f2 = float __attribute__((ext_vector_type(2)));
    auto adam_pair = [&](int q) {
        const f2 g = {gq[q], gq[q + 1]};
        const f2 gr = g * a_coef;
        f2 mm = {m[q], m[q + 1]}, vv = {v[q], v[q + 1]};
        const f2 c1 = ar1, c2 = ar2;
        mm = __builtin_elementwise_fma(c1, gr - mm, mm);
        vv = __builtin_elementwise_fma(c2, gr * gr, vv * hp.beta2);
        const f2 sq = {__builtin_amdgcn_sqrtf(vv.x), __builtin_amdgcn_sqrtf(vv.y)};
        const f2 den = __builtin_elementwise_fma(sq, (f2)a_ib, (f2)hp.eps);
        const f2 r = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
        const f2 wv = {wq[q], wq[q + 1]};
        const f2 wn = __builtin_elementwise_fma((f2)(-a_ss), mm * r, wv);
        m[q] = mm.x;
        m[q + 1] = mm.y;
        v[q] = vv.x;
        v[q + 1] = vv.y;
        W[lp[q]] = wn.x;
        W[lp[q + 1]] = wn.y;
    };
    // slots [q0, q1) of this thread's Adam step (pairs when kPK)
    auto adam_slots = [&](auto q0c, auto q1c) {
        constexpr int q0 = decltype(q0c)::value, q1 = decltype(q1c)::value;
        if constexpr (kPK) {
            static_assert(q0 % 2 == 0 && q1 % 2 == 0, "packed Adam runs slot pairs");
#pragma unroll
            for (int q = q0; q < q1; q += 2) adam_pair(q);
        } else {
#pragma unroll
            for (int q = q0; q < q1; ++q) adam_slot(q);
        }
    };
    // the deferred slots of the previous minibatch's Adam step (kAS)
    auto adam_rest = [&]() {
        adam_slots(std::integral_constant<int, kKA>{}, std::integral_constant<int, KP>{});
    };
    int64_t kmb = 0;
    for (int ep = 0; ep < g.n_epochs; ++ep) {
        for (int64_t s0 = 0; s0 < n; s0 += bs, ++kmb) {
            const int B = (int)((n - s0) < bs ? (n - s0) : bs);
            // loss means: over this minibatch, or (gradient mode) over the global minibatch
            const float invB = GRAD ? g.inv_bg : 1.0f / (float)B;
            float gss = 0.f;  // sum of squares of the gradient entries this thread writes
            // ---- gather the minibatch (from the prefetch registers), then start the next one
            // (late gather: this minibatch's rows were stored at the end of the previous one)
            if (!kLate || kmb == 0) gather_store(B, (SPLIT && net_b == 0) ? adv_nx : ps[3]);
            load_rows(ro_n, rs_n, po, ps);
            perm_rows(e2, s2, ro_n, rs_n);
            advance(e2, s2);
            if (!kLate || kmb == 0) __syncthreads();
            FENV_PPO_PHASE(0);
            // ---- advantage normalisation (wave 0) || layer 1 (all waves)
            if (!SPLIT && w == 0 && hp.normalize_advantage && B > 1) {
                const float a = lane < B ? S[sADV * kPB + lane] : 0.0f;
                const float mean = wsum(a) * invB;
                const float d = lane < B ? a - mean : 0.0f;
                const float sd = __builtin_sqrtf(wsum(d * d) / (float)(B - 1));
                if (lane < B) S[sADV * kPB + lane] = (a - mean) / (sd + 1e-8f);
            }
            // layer 1 on v_mfma_f32_16x16x4f32: wave w = net w>>2, hidden units 16(w&3)..+15, all
            // 64 sample rows as 4 tiles; K = 8 obs columns (zero-padded past D) as 2 MFMAs.  The
            // W1 operand past column D reads the next row's weights, multiplied by O's zeros.
            auto layer1 = [&]() {
                const int net = w >> 2, jt = w & 3, q = lane >> 4, c = lane & 15;
                const int j = 16 * jt + c;
                const int w1 = (net ? L.vf0W : L.pi0W) + j * D + q;
                const float b0 = W[lx(w1)], b1 = W[lx(w1 + 4)];
                const float bias = W[lx((net ? L.vf0b : L.pi0b) + j)];
                // the 4 tiles' observation operands read up front (one LDS wait for the phase
                // instead of one per tile)
                float oa[4], ob[4];
#pragma unroll
                for (int bt = 0; bt < 4; ++bt) {
                    const float *o = O + (16 * bt + c) * 9 + q;
                    oa[bt] = o[0];
                    ob[bt] = o[4];
                }
#pragma unroll
                for (int bt = 0; bt < 4; ++bt) {
                    f32x4 acc = {bias, bias, bias, bias};
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(oa[bt], b0, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ob[bt], b1, acc, 0, 0, 0);
                    float *hr = H1 + (net * kPB + 16 * bt + 4 * q) * kRow + j;
#pragma unroll
                    for (int r = 0; r < 4; r += 2) {
                        float y0, y1;
                        tanh_u2(acc[r], acc[r + 1], y0, y1);
                        hr[r * kRow] = y0;
                        hr[(r + 1) * kRow] = y1;
                    }
                }
            };
            // kAS: the previous minibatch's deferred Adam slots in the same straight-line block
            // as layer 1 (one basic block, so the two interleave)
            if (kAS && kmb > 0) {
                layer1();
                adam_rest();
            } else {
                layer1();
            }
            __syncthreads();
            FENV_PPO_PHASE(1);
            // the loss's log_std-derived constants (formed by every wave in the heads phase)
            float lc_var0 = 0.f, lc_var1 = 0.f, lc_lsd0 = 0.f, lc_lsd1 = 0.f;
            float lc_i2v0 = 0.f, lc_i2v1 = 0.f, lc_iv0 = 0.f, lc_iv1 = 0.f;
            auto loss_consts = [&]() {
                const float ls0 = W[lx(L.logstd)], ls1 = W[lx(L.logstd + 1)];
                // the loss wave's chain starts from these: hardware exp / log / reciprocal
                // (v_exp_f32, v_log_f32, v_rcp_f32: ~1 ulp) instead of libm expf / logf and
                // correctly rounded divisions (~70 dependent instructions)
                const float kL2e = 1.44269504088896341f, kLn2 = 0.693147180559945309f;
                const float sd0 = __builtin_amdgcn_exp2f(ls0 * kL2e);
                const float sd1 = __builtin_amdgcn_exp2f(ls1 * kL2e);
                lc_var0 = sd0 * sd0;
                lc_var1 = sd1 * sd1;
                lc_lsd0 = __builtin_amdgcn_logf(sd0) * kLn2;  // torch: std.log()
                lc_lsd1 = __builtin_amdgcn_logf(sd1) * kLn2;
                lc_iv0 = __builtin_amdgcn_rcpf(lc_var0);
                lc_iv1 = __builtin_amdgcn_rcpf(lc_var1);
                lc_i2v0 = 0.5f * lc_iv0;
                lc_i2v1 = 0.5f * lc_iv1;
            };
            // ---- layer 2: wave w = one 32 x 32 tile (net w>>2, sample rows 32((w>>1)&1), hidden
            // cols 32(w&1)) of Z2 = b2 + H1 . W2^T, K = 64 as four 16-deep split-f16 chunks
            // (12 v_mfma_f32_32x32x16_f16 instead of 32 fp32 32x32x2: round 4, 8.60-8.74 ->
            // 8.21-8.29 us per minibatch with this phase alone).  Every row runs (rows >= B unused).
            {
                const int net = w >> 2, mt = (w >> 1) & 1, nt = w & 1, h = lane >> 5;
                const int c = lane & 31;
                const float *Ar = H1 + (net * kPB + 32 * mt + c) * kRow + 32 * h;
                const float *Bc = W + lx(net ? L.vf2W : L.pi2W) + (32 * nt + c) * kRow + 32 * h;
                const float bias = W[lx((net ? L.vf2b : L.pi2b) + 32 * nt + c)];
                f32x16 acc;
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = bias;
                // lane half h carries k = 32h + 8cc + j of chunk cc; small terms first
                float av[4][8], bv[4][8];
#pragma unroll
                for (int cc = 0; cc < 4; ++cc)
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        av[cc][j] = Ar[8 * cc + j];
                        bv[cc][j] = Bc[8 * cc + j];
                    }
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) {
                    h8 ah, al, bh, bl;
                    split8(av[cc], 0, ah, al);
                    split8(bv[cc], 0, bh, bl);
                    acc = mma16(ah, bl, acc);
                    acc = mma16(al, bh, acc);
                    acc = mma16(ah, bh, acc);
                }
                float *Hr = H2 + (net * kPB + 32 * mt) * kRow + 32 * nt + c;
#pragma unroll
                for (int r = 0; r < 16; r += 2) {
                    float y0, y1;
                    tanh_u2(acc[r], acc[r + 1], y0, y1);
                    Hr[rho(r, h) * kRow] = y0;
                    Hr[rho(r + 1, h) * kRow] = y1;
                }
            }
            __syncthreads();
            // ---- heads mu = actW . h2_pi + actb, value = valW . h2_vf + valb on
            // v_mfma_f32_16x16x4f32: wave w = net w>>2, samples 16(w&3)..+15, output columns 0..15
            // of which 2 (actor) / 1 (critic) are real; K = 64 hidden as 16 MFMAs
            // The loss constants are formed here, in this phase's MFMA shadow (every wave), off the
            // loss wave's dependent chain (round 4, with the hardware-exp ratio and the late loss
            // sums: 7.83 -> 7.72 us per minibatch, profiles/ab/r4_ppo_loss_phase_ab.txt)
            loss_consts();
            {
                const int net = w >> 2, bt = w & 3, q = lane >> 4, c = lane & 15;
                const int ncol = net ? 1 : 2;
                const float *a = H2 + (net * kPB + 16 * bt + c) * kRow + q;
                const int hw = net ? L.valW : L.actW + (c & 1) * kHid;
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
                if constexpr (SPLIT) {  // operands read up front, branch-free (see head grads)
                    // K-step s4 of lane group q: hidden unit 16 q + s4 (the 64 lanes of a read hit
                    // 64 banks)
                    float av[16], wv[16];
#pragma unroll
                    for (int s4 = 0; s4 < 16; ++s4) {
                        const int kk = 16 * q + s4;
                        av[s4] = a[kk - q];
                        wv[s4] = W[lx(hw + kk)];
                    }
                    f32x4 acc2 = {0.f, 0.f, 0.f, 0.f};  // kAcc2: two chains (even / odd steps)
#pragma unroll
                    for (int s4 = 0; s4 < 16; ++s4) {
                        const float bw = c < ncol ? wv[s4] : 0.0f;
                        if (kAcc2 && (s4 & 1))
                            acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s4], bw, acc2, 0, 0, 0);
                        else
                            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s4], bw, acc, 0, 0, 0);
                    }
                    if (kAcc2)
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc[r] += acc2[r];
                } else {
#pragma unroll
                    for (int s4 = 0; s4 < 16; ++s4) {
                        const float bw = c < ncol ? W[lx(hw + 4 * s4 + q)] : 0.0f;
                        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[4 * s4], bw, acc, 0, 0, 0);
                    }
                }
                if (c < ncol) {
                    const float hb = W[lx(net ? L.valb : L.actb + c)];
                    float *so = S + (net ? sVAL : sMU0 + c) * kPB + 16 * bt + 4 * q;
#pragma unroll
                    for (int r = 0; r < 4; ++r) so[r] = acc[r] + hb;
                }
            }
            __syncthreads();
            FENV_PPO_PHASE(2);
            // ---- heads, losses and per-sample gradients (wave 0, lane = sample; split: wave 0 of
            // each block, the actor block keeping the policy/entropy terms, the critic block the
            // value terms)
            if (wl == 0) {
                const bool do_pi = !SPLIT || net_b == 0, do_vf = !SPLIT || net_b == 1;
                const bool on = lane < B;
                const float lsd0 = lc_lsd0, lsd1 = lc_lsd1, i2v0 = lc_i2v0, i2v1 = lc_i2v1;
                const float iv0 = lc_iv0, iv1 = lc_iv1;
                float pl = 0.f, vl = 0.f, cf = 0.f, gls0 = 0.f, gls1 = 0.f, gmu0 = 0.f, gmu1 = 0.f;
                float gv = 0.f;
                if constexpr (kSpread) {
                    // split launch: this block's terms only; the sums over the samples are taken
                    // after the barrier (loss_sums, loss_stats; per-sample values in S)
                    const float kLogSqrt2Pi = 0.918938533204672742f;
                    if (do_pi) {
                        if (on) {
                            const float mu0 = S[sMU0 * kPB + lane], mu1 = S[sMU1 * kPB + lane];
                            const float a0 = S[sA0 * kPB + lane], a1 = S[sA1 * kPB + lane];
                            const float d0 = a0 - mu0, d1 = a1 - mu1;
                            const float lp = (-(d0 * d0) * i2v0 - lsd0 - kLogSqrt2Pi) +
                                             (-(d1 * d1) * i2v1 - lsd1 - kLogSqrt2Pi);
                            // v_exp_f32 on a log2(e) product (~2 ulp for the |log ratio| < 1 that
                            // stays unclipped) instead of libm expf's range-reduced form
                            const float ratio = __builtin_amdgcn_exp2f(
                                (lp - S[sOLP * kPB + lane]) * 1.44269504088896341f);
                            const float an = S[sADV * kPB + lane];
                            const float lo = 1.0f - hp.clip_range, hi = 1.0f + hp.clip_range;
                            const float rc = ratio < lo ? lo : (ratio > hi ? hi : ratio);
                            const float l1 = an * ratio, l2 = an * rc;
                            pl = l1 < l2 ? l1 : l2;
                            cf = fabsf(ratio - 1.0f) > hp.clip_range ? 1.0f : 0.0f;
                            const float g1 = l1 < l2 ? 1.0f : (l1 == l2 ? 0.5f : 0.0f);
                            const float g2 = l2 < l1 ? 1.0f : (l1 == l2 ? 0.5f : 0.0f);
                            const float inside = (ratio >= lo && ratio <= hi) ? 1.0f : 0.0f;
                            const float dratio = -(g1 * an + g2 * an * inside) * invB;
                            const float dlp = dratio * ratio;
                            gmu0 = dlp * (d0 * iv0);
                            gmu1 = dlp * (d1 * iv1);
                            gls0 = dlp * ((d0 * d0) * iv0 - 1.0f);
                            gls1 = dlp * ((d1 * d1) * iv1 - 1.0f);
                        }
                        S[sGMU0 * kPB + lane] = gmu0;
                        S[sGMU1 * kPB + lane] = gmu1;
                        S[sPL * kPB + lane] = pl;
                        S[sCF * kPB + lane] = cf;
                        S[sGL0 * kPB + lane] = gls0;
                        S[sGL1 * kPB + lane] = gls1;
                        if (lane == 0) {
                            const float kHalfLog2PiE = 1.41893853320467274f;  // 0.5 + 0.5 log(2 pi)
                            R[kEnt] = (kHalfLog2PiE + lsd0) + (kHalfLog2PiE + lsd1);
                        }
                    } else {
                        if (on) {
                            const float rr = S[sRET * kPB + lane] - S[sVAL * kPB + lane];
                            vl = rr * rr;
                            gv = hp.vf_coef * (-2.0f * rr) * invB;
                        }
                        S[sGV * kPB + lane] = gv;
                        S[sVLS * kPB + lane] = vl;
                    }
                } else if (on) {
                    const float mu0 = S[sMU0 * kPB + lane], mu1 = S[sMU1 * kPB + lane];
                    const float val = S[sVAL * kPB + lane];
                    const float a0 = S[sA0 * kPB + lane], a1 = S[sA1 * kPB + lane];
                    const float d0 = a0 - mu0, d1 = a1 - mu1;
                    const float kLogSqrt2Pi = 0.918938533204672742f;
                    // divisions by 2 var and var as products with their reciprocals (1 ulp)
                    const float lp = (-(d0 * d0) * i2v0 - lsd0 - kLogSqrt2Pi) +
                                     (-(d1 * d1) * i2v1 - lsd1 - kLogSqrt2Pi);
                    const float ratio = expf(lp - S[sOLP * kPB + lane]);
                    const float an = S[sADV * kPB + lane];
                    const float lo = 1.0f - hp.clip_range, hi = 1.0f + hp.clip_range;
                    const float rc = ratio < lo ? lo : (ratio > hi ? hi : ratio);
                    const float l1 = an * ratio, l2 = an * rc;
                    pl = l1 < l2 ? l1 : l2;
                    cf = fabsf(ratio - 1.0f) > hp.clip_range ? 1.0f : 0.0f;
                    const float rr = S[sRET * kPB + lane] - val;
                    vl = rr * rr;
                    // torch.minimum: ties split the gradient; clamp passes it inside [lo, hi]
                    const float g1 = l1 < l2 ? 1.0f : (l1 == l2 ? 0.5f : 0.0f);
                    const float g2 = l2 < l1 ? 1.0f : (l1 == l2 ? 0.5f : 0.0f);
                    const float inside = (ratio >= lo && ratio <= hi) ? 1.0f : 0.0f;
                    const float dratio = -(g1 * an + g2 * an * inside) * invB;
                    const float dlp = dratio * ratio;
                    gv = hp.vf_coef * (-2.0f * rr) * invB;
                    gmu0 = dlp * (d0 * iv0);
                    gmu1 = dlp * (d1 * iv1);
                    gls0 = dlp * ((d0 * d0) * iv0 - 1.0f);
                    gls1 = dlp * ((d1 * d1) * iv1 - 1.0f);
                }
                if constexpr (!kSpread) {
                if (do_pi) {
                    S[sGMU0 * kPB + lane] = gmu0;
                    S[sGMU1 * kPB + lane] = gmu1;
                }
                if (do_vf) S[sGV * kPB + lane] = gv;
                pl = wsum(pl);
                vl = wsum(vl);
                cf = wsum(cf);
                gls0 = wsum(gls0);
                gls1 = wsum(gls1);
                const float sgmu0 = wsum(gmu0), sgmu1 = wsum(gmu1), sgv = wsum(gv);
                if (lane == 0) {
                    gss = 0.0f;
                    if (do_pi) {
                        const float kHalfLog2PiE = 1.41893853320467274f;  // 0.5 + 0.5 log(2 pi)
                        const float ent = (kHalfLog2PiE + lsd0) + (kHalfLog2PiE + lsd1);
                        st_pl += (double)(-pl * invB);
                        if (!GRAD || g.ent_once) st_el += (double)(-ent);
                        st_cf += (double)(cf * invB);
                        // d(ent_coef * entropy_loss)/d log_std_j = -ent_coef (d log(exp(ls))/d ls
                        // = 1)
                        // gradient mode: the entropy term once over the ranks (ent_once)
                        const float ec = (!GRAD || g.ent_once) ? hp.ent_coef : 0.0f;
                        const float g0 = gls0 - ec, g1 = gls1 - ec;
                        G[lx(L.logstd)] = g0;
                        G[lx(L.logstd + 1)] = g1;
                        G[lx(L.actb)] = sgmu0;
                        G[lx(L.actb + 1)] = sgmu1;
                        gss = g0 * g0 + g1 * g1 + sgmu0 * sgmu0 + sgmu1 * sgmu1;
                    }
                    if (do_vf) {
                        st_vl += (double)(vl * invB);
                        G[lx(L.valb)] = sgv;
                        gss += sgv * sgv;
                    }
                }
                }  // !kSpread
            } else if (kBCW && wl == 1) {
                // kBCW: this minibatch's Adam bias corrections (they depend on the step count
                // only), by a wave that would otherwise wait out the loss at the barrier; every
                // thread reads them after the norm exchange instead of computing them there
                pw1 *= (double)hp.beta1;  // beta^(step + 1)
                pw2 *= (double)hp.beta2;
                const float bc1 = 1.0f - (float)pw1;
                const float bc2 = 1.0f - (float)pw2;
                const float ss = hp.lr / bc1, ib = 1.0f / __builtin_sqrtf(bc2);
                if (lane == 0) {
                    R[kBC] = ss;
                    R[kBC + 1] = ib;
                }
            }
            __syncthreads();
            FENV_PPO_PHASE(3);
            // kSpread: the loss sums.  The four actor gradient sums go one per wave (waves 0-3,
            // branch-free; the critic's value-bias sum to wave 2); the statistics sums (policy /
            // value loss, clip fraction) wait for the norm phase's exchange shadow (loss_stats),
            // except in gradient mode, which has no norm phase.  Their outputs are only read from
            // the norm phase on.
            auto loss_stats = [&]() {
                if (wl == 1) {
                    if (net_b == 0) {
                        const float spl = wsum(S[sPL * kPB + lane]), scf = wsum(S[sCF * kPB + lane]);
                        if (lane == 0) {
                            st_pl += (double)(-spl * invB);
                            if (!GRAD || g.ent_once) st_el += (double)(-R[kEnt]);
                            st_cf += (double)(scf * invB);
                        }
                    } else {
                        const float svl = wsum(S[sVLS * kPB + lane]);
                        if (lane == 0) st_vl += (double)(svl * invB);
                    }
                }
            };
            auto loss_sums = [&]() {
                if constexpr (GRAD) loss_stats();
                if (net_b == 0) {
                    // wave wl: d log_std_0, d log_std_1, d actb_0, d actb_1.  d(ent_coef *
                    // entropy_loss)/d log_std_j = -ent_coef; gradient mode: the entropy term once
                    // over the ranks (ent_once)
                    const float ec = (!GRAD || g.ent_once) ? hp.ent_coef : 0.0f;
                    const int slot = wl == 0 ? sGL0 : (wl == 1 ? sGL1 : (wl == 2 ? sGMU0 : sGMU1));
                    const int gi = wl < 2 ? L.logstd + wl : L.actb + (wl - 2);
                    const float v = wsum(S[slot * kPB + lane]) - (wl < 2 ? ec : 0.0f);
                    if (lane == 0) {
                        G[lx(gi)] = v;
                        gss += v * v;
                    }
                } else if (wl == 2) {
                    const float sgv = wsum(S[sGV * kPB + lane]);
                    if (lane == 0) {
                        G[lx(L.valb)] = sgv;
                        gss += sgv * sgv;
                    }
                }
            };
            if constexpr (kSpread) loss_sums();
            // ---- head weight gradients on v_mfma_f32_16x16x4f32 (wave w = net w>>2, hidden rows
            // 16(w&3)..+15, columns gmu0/gmu1 resp. gv; K = 64 samples as 16 MFMAs), then
            // dL/dz2 in place over the SAME H2 columns (only this wave reads or writes them in
            // this phase, so no barrier between); rows b >= B are zeroed so the contractions
            // over all 64 samples ignore them
            if constexpr (SPLIT) {
                // one wave per SIMD and a 512-register budget: every LDS operand of the phase is
                // read up front (one wait instead of one per step) and the dL/dz2 loop is
                // branch-free (rows b >= B select 0); same operations as the unsplit form below
                const int net = w >> 2, kt = w & 3, q = lane >> 4, c = lane & 15;
                const int ncol = net ? 1 : 2;
                float *hcol = H2 + net * kPB * kRow + 16 * kt;
                const float *sg = S + (net ? sGV : sGMU0 + (c & 1)) * kPB;
                const float *s0p = S + (net ? sGV : sGMU0) * kPB, *s1p = S + sGMU1 * kPB;
                float ha[16], sb[16], s0[16], s1[16];
                // sample of K-step t: b = 16 q + t (the per-sample scalars of a
                // lane group are then 16 contiguous floats, read as four ds_read_b128) or 4 t + q
                auto bidx = [&](int t) { return 16 * q + t; };
#pragma unroll
                for (int t = 0; t < 16; ++t) ha[t] = hcol[bidx(t) * kRow + c];
                {
                    const float4 *g4 = reinterpret_cast<const float4 *>(sg + 16 * q);
                    const float4 *a4 = reinterpret_cast<const float4 *>(s0p + 16 * q);
                    const float4 *c4 = reinterpret_cast<const float4 *>(s1p + 16 * q);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float4 x = g4[j], y = a4[j];
                        const float4 z = net ? make_float4(0.f, 0.f, 0.f, 0.f) : c4[j];
                        sb[4 * j] = x.x; sb[4 * j + 1] = x.y; sb[4 * j + 2] = x.z; sb[4 * j + 3] = x.w;
                        s0[4 * j] = y.x; s0[4 * j + 1] = y.y; s0[4 * j + 2] = y.z; s0[4 * j + 3] = y.w;
                        s1[4 * j] = z.x; s1[4 * j + 1] = z.y; s1[4 * j + 2] = z.z; s1[4 * j + 3] = z.w;
                    }
                }
                const int k = 16 * kt + c;
                const float wa0 = W[lx((net ? L.valW : L.actW) + k)];
                const float wa1 = net ? 0.0f : W[lx(L.actW + kHid + k)];
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
                f32x4 acc2 = {0.f, 0.f, 0.f, 0.f};  // kAcc2: two chains (even / odd steps)
#pragma unroll
                for (int t = 0; t < 16; ++t) {
                    const float bs_ = c < ncol ? sb[t] : 0.0f;
                    if (kAcc2 && (t & 1))
                        acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(ha[t], bs_, acc2, 0, 0, 0);
                    else
                        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ha[t], bs_, acc, 0, 0, 0);
                }
                if (kAcc2)
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[r] += acc2[r];
                float b2p = 0.0f;  // kB2: this lane's part of the b2 gradient of column k
                float zmx = 0.0f;  // max |dL/dz2| of the lane's entries (split-f16 W2 phase scale)
#pragma unroll
                for (int t = 0; t < 16; ++t) {
                    const int b = bidx(t);
                    const float gh = net ? s0[t] * wa0 : s0[t] * wa0 + s1[t] * wa1;
                    const float hv = ha[t];
                    const float dz = gh * (1.0f - hv * hv);
                    const float dzb = b < B ? dz : 0.0f;
                    hcol[b * kRow + c] = dzb;
                    if (kB2) b2p += dzb;
                    zmx = fmaxf(zmx, fabsf(dzb));
                }
                zmx = wmax_nn(zmx);
                if (lane == 0) R[kZM + w] = zmx;
                if constexpr (kB2) {  // b2 gradient = column sum of dL/dz2 (the 4 lane groups)
                    b2p += __shfl_xor(b2p, 16, 64);
                    b2p += __shfl_xor(b2p, 32, 64);
                    if (q == 0) {
                        G[lx((net ? L.vf2b : L.pi2b) + k)] = b2p;
                        gss = __builtin_fmaf(b2p, b2p, gss);
                    }
                }
                if (c < ncol) {
                    const int hw = net ? L.valW : L.actW + c * kHid;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        G[lx(hw + 16 * kt + 4 * q + r)] = acc[r];
                        gss = __builtin_fmaf(acc[r], acc[r], gss);
                    }
                }
            } else {
                const int net = w >> 2, kt = w & 3, q = lane >> 4, c = lane & 15;
                const int ncol = net ? 1 : 2;
                float *hcol = H2 + net * kPB * kRow + 16 * kt;
                const float *sg = S + (net ? sGV : sGMU0 + (c & 1)) * kPB;
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s4 = 0; s4 < 16; ++s4) {
                    const int b = 4 * s4 + q;
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(hcol[b * kRow + c],
                                                              c < ncol ? sg[b] : 0.0f, acc, 0, 0, 0);
                }
                if (c < ncol) {
                    const int hw = net ? L.valW : L.actW + c * kHid;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        G[lx(hw + 16 * kt + 4 * q + r)] = acc[r];
                        gss = __builtin_fmaf(acc[r], acc[r], gss);
                    }
                }
                const int k = 16 * kt + c;
                const float wa0 = W[lx((net ? L.valW : L.actW) + k)];
                const float wa1 = net ? 0.0f : W[lx(L.actW + kHid + k)];
                float zmx = 0.0f;
#pragma unroll FENV_PPO_UDZ
                for (int t = 0; t < 16; ++t) {
                    const int b = 4 * t + q;
                    float *hp2 = hcol + b * kRow + c;
                    float v = 0.0f;
                    if (b < B) {
                        const float gh = net ? S[sGV * kPB + b] * wa0
                                             : S[sGMU0 * kPB + b] * wa0 + S[sGMU1 * kPB + b] * wa1;
                        const float hv = *hp2;
                        v = gh * (1.0f - hv * hv);
                    }
                    *hp2 = v;
                    zmx = fmaxf(zmx, fabsf(v));
                }
                zmx = wmax_nn(zmx);
                if (lane == 0) R[kZM + w] = zmx;
            }
            __syncthreads();
            FENV_PPO_PHASE(4);
            FENV_PPO_PHASE(5);
            // ---- W2 gradients GW2 = dZ2^T . H1 and dL/dh1 = dZ2 . W2, both with K = 64 (samples b
            // resp. hidden j) as four 16-deep split-f16 chunks (round 4: 24 v_mfma_f32_32x32x16_f16
            // instead of 64 fp32 32x32x2; with layer 2, 8.60-8.74 -> 7.79-7.96 us per minibatch).
            // Wave w owns tile (net w>>2, rows 32((w>>1)&1), cols 32(w&1)) of each; dL/dz1
            // overwrites H1 only after the barrier (GW2 reads H1).
            {
                const int net = w >> 2, mt = (w >> 1) & 1, nt = w & 1, h = lane >> 5;
                const int c = lane & 31;
                const int w2 = lx(net ? L.vf2W : L.pi2W);
                const float *Z2 = H2 + net * kPB * kRow;  // dL/dz2 [b][j]
                const float *A1 = H1 + net * kPB * kRow;  // h1 [b][k]
                f32x16 gw, dz;
#pragma unroll
                for (int r = 0; r < 16; ++r) gw[r] = dz[r] = 0.0f;
                // kDZP: tanh' = 1 - h1^2 of this wave's dL/dz1 tile, read and formed before the
                // MFMA chains (h1 is read-only in this phase), so the tail after them is a product
                float omh[16];
                if constexpr (kDZP) {
                    const float *H1p = H1 + (net * kPB + 32 * mt) * kRow + 32 * nt + c;
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float hv = H1p[rho(r, h) * kRow];
                        omh[r] = 1.0f - hv * hv;
                    }
                }
                // split-f16 chains (three v_mfma_f32_32x32x16_f16 per 16-deep chunk, lane half h
                // carrying k = 32h + 8cc + j); dL/dz2 scaled by a power of two so its largest
                // entry sits at 2^10..2^11 in f16 (exact: the results are scaled back)
                const float *zmw = R + kZM + 4 * net;  // this network's four wave maxima
                const float zm = fmaxf(fmaxf(zmw[0], zmw[1]), fmaxf(zmw[2], zmw[3]));
                int se = 264 - (int)((__float_as_uint(zm) >> 23) & 0xFFu);  // 127 + 10 - e
                // <= 253 keeps the unscale factor 2^(127 - se) a normal number (254 made it +0
                // and zeroed the W2 / dL/dh1 gradients of a network whose max |dL/dz2| < 2^-116)
                se = se < 1 ? 1 : (se > 253 ? 253 : se);
                const float zs = __uint_as_float((uint32_t)se << 23);
                const float zi = __uint_as_float((uint32_t)(254 - se) << 23);
                const float *pa = Z2 + (32 * h) * kRow + 32 * mt + c;
                const float *pb = A1 + (32 * h) * kRow + 32 * nt + c;
                const float *pc = Z2 + (32 * mt + c) * kRow + 32 * h;
                const float *pd = W + w2 + (32 * h) * kRow + 32 * nt + c;
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) {
                    float va[8], vb[8], vc[8], vd[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int i = 8 * cc + j;
                        va[j] = pa[i * kRow] * zs;
                        vb[j] = pb[i * kRow];
                        vc[j] = pc[i] * zs;
                        vd[j] = pd[i * kRow];
                    }
                    h8 ah, al, bh, bl, ch, cl, dh, dl;
                    split8(va, 0, ah, al);
                    split8(vb, 0, bh, bl);
                    split8(vc, 0, ch, cl);
                    split8(vd, 0, dh, dl);
                    gw = mma16(ah, bl, gw);
                    dz = mma16(ch, dl, dz);
                    gw = mma16(al, bh, gw);
                    dz = mma16(cl, dh, dz);
                    gw = mma16(ah, bh, gw);
                    dz = mma16(ch, dh, dz);
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    gw[r] *= zi;
                    dz[r] *= zi;
                }
                float *Gr = G + w2 + 32 * mt * kRow + 32 * nt + c;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    Gr[rho(r, h) * kRow] = gw[r];
                    gss = __builtin_fmaf(gw[r], gw[r], gss);
                }
                if (!kB2 && tid < (SPLIT ? kHid : 2 * kHid)) {
                    const int bn = SPLIT ? net_b : tid >> 6, j = tid & 63;
                    const float *z2 = H2 + bn * kPB * kRow + j;
                    const float acc = col_sum(z2, B);
                    G[lx((bn ? L.vf2b : L.pi2b) + j)] = acc;
                    gss = __builtin_fmaf(acc, acc, gss);
                }
                // kZ1S: dL/dz1 goes to the other network's (unused) H1 half, so no wave's write can
                // overtake another wave's GW2 reads of h1 and no barrier is needed here
                if (!kZ1S) __syncthreads();
                FENV_PPO_PHASE(6);
                const float *H1r = H1 + (net * kPB + 32 * mt) * kRow + 32 * nt + c;
                float *Z1w = H1 + ((kZ1S ? zb : net) * kPB + 32 * mt) * kRow + 32 * nt + c;
                float b1p = 0.0f;  // kB1: this lane's part of the b1 gradient of its column
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float hv = kDZP ? 0.0f : H1r[rho(r, h) * kRow];
                    const float z1 = kDZP ? dz[r] * omh[r] : dz[r] * (1.0f - hv * hv);
                    Z1w[rho(r, h) * kRow] = z1;
                    if (kB1) b1p += z1;
                }
                if constexpr (kB1) {  // rows of this tile (both lane halves); the other row tile's
                    b1p += __shfl_xor(b1p, 32, 64);  // wave adds its part in the W1 phase
                    if (h == 0) B1P[mt * kHid + 32 * nt + c] = b1p;
                }
            }
            __syncthreads();
            FENV_PPO_PHASE(7);
            // ---- W1 gradients GW1 = dZ1^T . O on v_mfma_f32_16x16x4f32 (wave w: net w>>2, hidden
            // rows 16(w&3)..+15, obs columns 0..15 of which 0..D-1 are real; K = 64 samples,
            // slot q <-> sample 16q + i) and b1 gradients
            {
                const int net = w >> 2, jt = w & 3, q = lane >> 4, c = lane & 15;
                const float *Z1 = H1 + (kZ1S ? zb : net) * kPB * kRow + 16 * jt + c;
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
                if constexpr (SPLIT) {  // operands read up front, branch-free (see head grads)
                    float zv[16], ov[16];
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int b = 16 * q + i;
                        zv[i] = Z1[b * kRow];
                        ov[i] = O[b * 9 + (c & 7)];
                    }
                    f32x4 acc2 = {0.f, 0.f, 0.f, 0.f};  // kAcc2: two chains (even / odd steps)
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const float ob = c < 8 ? ov[i] : 0.0f;
                        if (kAcc2 && (i & 1))
                            acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(zv[i], ob, acc2, 0, 0, 0);
                        else
                            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(zv[i], ob, acc, 0, 0, 0);
                    }
                    if (kAcc2)
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc[r] += acc2[r];
                } else {
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int b = 16 * q + i;
                        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(Z1[b * kRow],
                                                                  c < 8 ? O[b * 9 + c] : 0.0f, acc,
                                                                  0, 0, 0);
                    }
                }
                if (c < D) {
                    const int w1 = (net ? L.vf0W : L.pi0W) + (16 * jt + 4 * q) * D + c;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        G[lx(w1 + r * D)] = acc[r];
                        gss = __builtin_fmaf(acc[r], acc[r], gss);
                    }
                }
            }
            if (tid < (SPLIT ? kHid : 2 * kHid)) {
                const int net = SPLIT ? net_b : tid >> 6, j = tid & 63;
                const float *z1 = H1 + (kZ1S ? (net ^ 1) : net) * kPB * kRow + j;
                const float acc = kB1 ? B1P[j] + B1P[kHid + j] : col_sum(z1, B);
                G[lx((net ? L.vf0b : L.pi0b) + j)] = acc;
                gss = __builtin_fmaf(acc, acc, gss);
            }
            if constexpr (GRAD) {  // this rank's share of the minibatch gradient, unclipped
                __syncthreads();
#pragma unroll
                for (int q = 0; q < KP; ++q) {
                    const int p = own(q);
                    if (p < P) g.grad[p] = G[lx(p)];
                }
                continue;
            }
            // ---- clip_grad_norm_(max_grad_norm): global 2-norm from the squares each thread
            // accumulated as it wrote its gradient entries (every entry is written exactly once
            // per minibatch), one wave sum each, reduced after the barrier
            gss = wsum(gss);
            if (lane == 0) R[wl] = gss;
            __syncthreads();
            FENV_PPO_PHASE(8);
            // split: this thread's gradient and parameter entries are read right after the post
            // of the norm exchange below, so the LDS reads overlap its wait (not before it: LDS
            // reads complete in order, so 40 reads queued ahead of the partial's own would delay
            // the post)
            auto read_gw = [&]() {
                if constexpr (SPLIT) {
#pragma unroll
                    for (int q = 0; q < KP; ++q) {
                        gq[q] = G[lp[q]];
                        wq[q] = W[lp[q]];
                    }
                }
            };
                        float tot = 0.f;
            for (int q = 0; q < NT / 64; ++q) tot += R[q];
            if (SPLIT) {
                // the other network's partial (actor's first in the sum on both blocks).  The
                // wait is bounded: a missing partner poisons the update with NaN instead of
                // hanging the GPU.
                const uint64_t seq = (uint64_t)(kmb + 1);
                uint64_t o = 0;
                if (tid == 0) {
                    // one 64-bit word carries both the value and its sequence number, so relaxed
                    // device-scope atomics suffice (nothing else is published through it)
                    // two words per block, by minibatch parity: the partner's word for this
                    // minibatch cannot be overwritten before this block has read it (its next
                    // post to the same word is two minibatches on, which waits on this block)
                    if (!(g.inject_lost && net_b == 1))
                    __hip_atomic_store(g.xch + 2 * net_b + (kmb & 1),
                                       (seq << 32) | __float_as_uint(tot), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    if (!partner_lost) {
                        o = __hip_atomic_load(g.xch + 2 * (net_b ^ 1) + (kmb & 1),
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                read_gw();
                if constexpr (kSpread && !GRAD) loss_stats();
                // the actor's wave 0 normalises the next minibatch's advantages (loaded into ps
                // at this minibatch's gather) while the first load is in flight
                if (net_b == 0 && wl == 0 && kmb + 1 < nmb) {
                    const int64_t s1 = s0 + bs < n ? s0 + bs : 0;  // next minibatch's start
                    adv_nx = adv_norm((int)((n - s1) < bs ? (n - s1) : bs), ps[3]);
                }
                if constexpr (kLate) {  // the next minibatch's rows, under the exchange wait
                    if (kmb + 1 < nmb) {
                        const int64_t s1 = s0 + bs < n ? s0 + bs : 0;
                        gather_store((int)((n - s1) < bs ? (n - s1) : bs),
                                     net_b == 0 ? adv_nx : ps[3]);
                    }
                }
                if (tid == 0) {
                    // after one timed-out wait the partner is taken as lost for good: no further
                    // waits, so a broken launch ends in milliseconds, not one timeout per
                    // minibatch
                    const int max_spin = partner_lost ? 0 : (g.inject_lost ? (1 << 10) : (1 << 22));
                    for (int spin = 0; spin < max_spin && (o >> 32) != seq; ++spin) {
                        __builtin_amdgcn_s_sleep(1);
                        o = __hip_atomic_load(g.xch + 2 * (net_b ^ 1) + (kmb & 1),
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    partner_lost = (o >> 32) != seq;
                    const float other = partner_lost ? __builtin_nanf("") : __uint_as_float((uint32_t)o);
                    R[32] = net_b == 0 ? tot + other : other + tot;
                }
                __syncthreads();
                tot = R[32];
            }
            FENV_PPO_PHASE(9);
            // v_sqrt_f32 and v_rcp_f32 (1 ulp each) instead of the correctly
            // rounded square root and division (~25 dependent instructions after the exchange)
            const float norm = __builtin_amdgcn_sqrtf(tot);
            float coef = hp.max_grad_norm * __builtin_amdgcn_rcpf(norm + 1e-6f);
            coef = coef < 1.0f ? coef : 1.0f;
            // ---- Adam (torch semantics: lerp first moment, bias-corrected step)
            a_coef = coef;
            if constexpr (kBCW) {
                step += 1.0f;
                a_ss = R[kBC];
                a_ib = R[kBC + 1];
            } else {
                step += 1.0f;
                pw1 *= (double)hp.beta1;
                pw2 *= (double)hp.beta2;
                const float bc1 = 1.0f - (float)pw1;
                const float bc2 = 1.0f - (float)pw2;
                a_ss = hp.lr / bc1;
                a_ib = 1.0f / __builtin_sqrtf(bc2);
            }
            // kAS: slots 0..kKA-1 (layer 1) now, the rest in the next minibatch's layer-1 phase
            adam_slots(std::integral_constant<int, 0>{}, std::integral_constant<int, kKA>{});
            __syncthreads();
            FENV_PPO_PHASE(10);
        }
    }
    if constexpr (kAS) {  // the last minibatch's deferred Adam slots
        if (kmb > 0) adam_rest();
        __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < KP; ++q) {
        const int p = own(q);
        if (!GRAD && p < P) g.params[p] = W[lx(p)];
    }
#pragma unroll
    for (int q = 0; q < KP; ++q) {
        const int p = own(q);
        if (!GRAD && p < P) {
#if FENV_PPO_DUMP_GRAD  // diagnostic build: the last minibatch's unclipped gradient, its
                        // observations and dL/dz1 rows
            g.exp_avg[p] = G[lx(p)];
            g.exp_avg_sq[p] = p < kPB * 9 ? O[p] : (p < kPB * 9 + 2 * kPB * kHid
                ? H1[((p - kPB * 9) >> 6) * kRow + ((p - kPB * 9) & 63)] : 0.0f);
#else
            g.exp_avg[p] = m[q];
            g.exp_avg_sq[p] = v[q];
#endif
        }
    }
    if (tid == 0 && net_b == 0 && !GRAD) g.step[0] = step;
    if (tid == stat_tid && net_b == 0) {
        atomicAdd(g.stats + 0, st_pl);  // atomic: the other block may mark a lost exchange
        if (!SPLIT) g.stats[1] += st_vl;
        g.stats[2] += st_el;
        atomicAdd(g.stats + 3, st_cf);
    }
#if FENV_PPO_PROFILE  // 1: the actor block's phases, 2: the critic block's (split launch)
    if (tid == 0 && net_b == (FENV_PPO_PROFILE == 2 ? 1 : 0))
        for (int q = 0; q < 11; ++q) g.stats[4 + q] += prof[q];
#endif
    if (SPLIT && tid == stat_tid && net_b == 1) g.stats[1] += st_vl;
    // split: a norm exchange that timed out leaves NaN parameters; say so in the stats, which the
    // host checks (ppo.py).  Atomic adds, so the mark survives in whichever order the two blocks
    // write: NaN policy-loss sum, and a clip-fraction sum far below zero (a lost partner, not
    // divergence)
    if (SPLIT && tid == 0 && partner_lost) {
        atomicAdd(g.stats + 0, (double)__builtin_nanf(""));
        atomicAdd(g.stats + 3, -1e30);
    }
}

// clip_grad_norm_ + Adam over the (all-reduced) gradient of a data-parallel minibatch
// (ppo_apply): torch semantics, in torch's capturable-Adam operation order
// (torch/optim/adam.py _single_tensor_adam, capturable branch).  One workgroup: the 2-norm is
// summed in a fixed order (thread k: elements k, k + NT, ...; then a fixed tree).
constexpr int kAT = 1024;
__global__ __launch_bounds__(kAT) void k_ppo_apply(float *params, float *exp_avg,
                                                   float *exp_avg_sq, float *step,
                                                   const float *grad, int P, ppo_hparams hp,
                                                   float omb1, float omb2) {
    __shared__ float red[kAT / 64];
    __shared__ float s_coef, s_step, s_bc1, s_bc2;
    const int tid = threadIdx.x;
    float ss = 0.f;
    for (int p = tid; p < P; p += kAT) ss = __builtin_fmaf(grad[p], grad[p], ss);
    ss = wsum(ss);
    if ((tid & 63) == 0) red[tid >> 6] = ss;
    __syncthreads();
    if (tid == 0) {
        float tot = 0.f;
        for (int k = 0; k < kAT / 64; ++k) tot += red[k];
        const float norm = __builtin_sqrtf(tot);
        const float c = hp.max_grad_norm / (norm + 1e-6f);
        s_coef = c < 1.0f ? c : 1.0f;
        s_step = step[0] + 1.0f;
        step[0] = s_step;
        // 1 - beta^step, beta^step the correctly rounded fp32 power (torch's _foreach_pow)
        s_bc1 = 1.0f - (float)pow((double)hp.beta1, (double)s_step);
        s_bc2 = 1.0f - (float)pow((double)hp.beta2, (double)s_step);
    }
    __syncthreads();
    const float coef = s_coef;
    const float bc1 = s_bc1, bc2 = s_bc2;
    const float step_size = hp.lr / bc1, ssn = -step_size;
    const float bc2s = __builtin_sqrtf(bc2);
    for (int p = tid; p < P; p += kAT) {
        const float gr = grad[p] * coef;
        const float m = exp_avg[p] + omb1 * (gr - exp_avg[p]);  // lerp_, weight < 0.5
        const float v = exp_avg_sq[p] * hp.beta2 + omb2 * gr * gr;  // mul_ + addcmul_
        exp_avg[p] = m;
        exp_avg_sq[p] = v;
        const float denom = __builtin_sqrtf(v) / (bc2s * ssn) + hp.eps / ssn;
        params[p] = params[p] + m / denom;  // addcdiv_
    }
}

static hipError_t ppo_smem_attr(const void *fn) {
    // once per (kernel, device): hipFuncSetAttribute is device-scoped
    static std::mutex mu;
    static std::set<std::pair<const void *, int>> done;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(mu);
    if (done.count({fn, dev})) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPPOLdsBytes);
    if (e == hipSuccess) done.insert({fn, dev});
    return e;
}

static bool split_fits(int32_t D) {
    const PLayout L(D);
    return (L.vf0W - L.pi0W) + (L.valW - L.actW) + 2 <= kPTS * kPerTS &&
           (L.actW - L.vf0W) + (L.logstd - L.valW) <= kPTS * kPerTS;
}

size_t ppo_workspace_bytes_impl() { return 4 * sizeof(uint64_t); }

// test hook: the next n fused-update launches (any device / thread) lose their norm exchange
static std::atomic<int> g_inject_lost{0};
void ppo_set_inject(int n) { g_inject_lost.store(n < 0 ? 0 : n); }
static int ppo_take_inject() {
    int v = g_inject_lost.load();
    while (v > 0 && !g_inject_lost.compare_exchange_weak(v, v - 1)) {
    }
    return v > 0 ? 1 : 0;
}

hipError_t launch_ppo_update(float *params, float *exp_avg, float *exp_avg_sq, float *step,
                             int32_t D, const float *obs, const float *act,
                             const float *old_log_prob, const float *adv, const float *ret,
                             int64_t n, const int64_t *perm, int32_t n_epochs,
                             int32_t batch_size, const ppo_hparams &hp, double *stats,
                             void *workspace, hipStream_t st) {
    constexpr bool split = FENV_PPO_SPLIT != 0;
    hipError_t e = ppo_smem_attr(reinterpret_cast<const void *>(&k_ppo_update<split>));
    if (e != hipSuccess) return e;
    uint64_t *xch = nullptr;
    bool own_ws = false;
    if (split) {
        if (!split_fits(D)) return hipErrorInvalidValue;
        // the exchange words: the caller's workspace (one per PPO instance), or, without one, a
        // stream-ordered allocation for this launch only -- never shared between launches that
        // may run concurrently.  Cleared on the launch's stream (sequence numbers restart at 1).
        xch = static_cast<uint64_t *>(workspace);
        if (!xch) {
            e = hipMallocAsync(reinterpret_cast<void **>(&xch), ppo_workspace_bytes_impl(), st);
            if (e != hipSuccess) return e;
            own_ws = true;
        }
        e = hipMemsetAsync(xch, 0, ppo_workspace_bytes_impl(), st);
        if (e != hipSuccess) return e;
    }
    PPOArgs g{params, exp_avg, exp_avg_sq, step, obs, act, old_log_prob, adv, ret, perm, n,
              D, n_epochs, batch_size, hp, stats, xch, nullptr, 0.f, 0.f, 1.f, 0, 1,
              split ? ppo_take_inject() : 0};
    adam_rates(hp, g.omb1, g.omb2);
    if (split) {
        // A cooperative launch: the runtime admits the grid only when all 9 workgroups are
        // resident at once, so the actor and critic blocks cannot wait for a partner that is
        // queued behind other work (the bounded spin remains as a guard, and the inject hook
        // still exercises it).  Blocks 0 and 8 work; the dispatcher's round-robin puts them on
        // one XCD, so their exchange words stay in that XCD's L2.
        void *args[] = {&g};
        e = hipLaunchCooperativeKernel(reinterpret_cast<const void *>(&k_ppo_update<true>),
                                       dim3(9), dim3(kPTS), args, (unsigned)kPPOLdsBytes, st);
        if (e != hipSuccess) {
            if (own_ws) (void)hipFreeAsync(xch, st);
            return e;
        }
    } else
        hipLaunchKernelGGL(k_ppo_update<false>, dim3(1), dim3(kPT), kPPOLdsBytes, st, g);
    e = hipGetLastError();
    if (own_ws) {
        const hipError_t ef = hipFreeAsync(xch, st);
        if (e == hipSuccess) e = ef;
    }
    return e;
}

hipError_t launch_ppo_grad(const float *params, int32_t D, const float *obs, const float *act,
                           const float *old_log_prob, const float *adv, const float *ret,
                           const int64_t *rows, int32_t b_local, int32_t b_global,
                           float adv_mean, float adv_std, int32_t adv_normalize,
                           int32_t entropy_term, const ppo_hparams &hp, float *grad,
                           double *stats, hipStream_t st) {
    if (!split_fits(D)) return hipErrorInvalidValue;
    hipError_t e = ppo_smem_attr(reinterpret_cast<const void *>(&k_ppo_update<true, true>));
    if (e != hipSuccess) return e;
    PPOArgs g{const_cast<float *>(params), nullptr, nullptr, nullptr, obs, act, old_log_prob,
              adv, ret, rows, (int64_t)b_local, D, 1, b_local, hp, stats, nullptr, grad,
              1.0f / (float)b_global, adv_mean, adv_std,
              (adv_normalize && b_global > 1) ? 1 : 0, entropy_term ? 1 : 0, 0};
    adam_rates(hp, g.omb1, g.omb2);
    hipLaunchKernelGGL((k_ppo_update<true, true>), dim3(9), dim3(kPTS), kPPOLdsBytes, st, g);
    return hipGetLastError();
}

hipError_t launch_ppo_apply(float *params, float *exp_avg, float *exp_avg_sq, float *step,
                            const float *grad, int32_t D, const ppo_hparams &hp,
                            hipStream_t st) {
    const PLayout L(D);
    float omb1, omb2;
    adam_rates(hp, omb1, omb2);
    hipLaunchKernelGGL(k_ppo_apply, dim3(1), dim3(kAT), 0, st, params, exp_avg, exp_avg_sq, step,
                       grad, L.total, hp, omb1, omb2);
    return hipGetLastError();
}

}  // namespace fenvk
