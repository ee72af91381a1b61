// C-ABI host layer of libfenv.so (include/fenv.h): handle lifecycle, the reference's global
// MT19937 reset stream (torch.manual_seed + torch.rand, simulate.py:125,133,140) replayed on the
// host and staged to HBM, launch splitting at reset events, and error reporting.
#pragma clang fp contract(off)

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <new>
#include <thread>
#include <unordered_set>
#include <vector>

#include "fenv.h"
#include "fenv_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define FENV_HIP(expr)                                                                  \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(FENV_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// MT19937 (Matsumoto & Nishimura 1998; init_genrand seeding, as torch's CPU generator after
// torch.manual_seed and as std::mt19937), producing the same sequence as std::mt19937 but
// twisting the 624-word state a block at a time and tempering runs of it straight into the
// caller's buffer (`fill`), in loops the compiler vectorises, and skipping whole blocks in
// discard without tempering them: a config-3 set with its tags takes ~1/3 of the host time
// of libstdc++'s per-draw generator (§9.2).  Pinned bit for bit to the oracle's
// MT19937 by tests/test_oracle_golden.py (fenv_host_reset_draws) and to the reference's draws
// by the golden fixtures.
// Host-only hot loops (the MT19937 replay) get an AVX2 clone beside the baseline x86-64 one,
// picked at load time by the CPU.  hipcc also runs a device pass over this file, which has no
// multiversioning (and emits none of these host functions).
#if defined(__HIP_DEVICE_COMPILE__)
#define FENV_HOST_CLONES
#else
#define FENV_HOST_CLONES __attribute__((target_clones("avx2", "default")))
#endif
class Mt19937 {
    static constexpr int kN = 624, kM = 397;
    uint32_t s_[kN];
    int pos_ = kN;
    static uint32_t tw(uint32_t a, uint32_t b, uint32_t m) {
        const uint32_t y = (a & 0x80000000u) | (b & 0x7FFFFFFFu);
        return m ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908B0DFu);
    }
    static uint32_t temper(uint32_t y) {
        y ^= y >> 11;
        y ^= (y << 7) & 0x9D2C5680u;
        y ^= (y << 15) & 0xEFC60000u;
        return y ^ (y >> 18);
    }
    FENV_HOST_CLONES void twist() {
        for (int i = 0; i < kN - kM; ++i) s_[i] = tw(s_[i], s_[i + 1], s_[i + kM]);
        for (int i = kN - kM; i < kN - 1; ++i) s_[i] = tw(s_[i], s_[i + 1], s_[i + kM - kN]);
        s_[kN - 1] = tw(s_[kN - 1], s_[0], s_[kM - 1]);
        pos_ = 0;
    }

  public:
    Mt19937() { seed(5489u); }
    void seed(uint32_t v) {
        s_[0] = v;
        for (int i = 1; i < kN; ++i)
            s_[i] = 1812433253u * (s_[i - 1] ^ (s_[i - 1] >> 30)) + (uint32_t)i;
        pos_ = kN;
    }
    // the next n draws into d[0..n), tempered straight from the state a block at a time
    FENV_HOST_CLONES void fill(uint32_t *d, size_t n) {
        while (n) {
            if (pos_ == kN) twist();
            const size_t k = std::min<size_t>(n, (size_t)(kN - pos_));
            const uint32_t *src = s_ + pos_;
            for (size_t i = 0; i < k; ++i) d[i] = temper(src[i]);
            d += k;
            n -= k;
            pos_ += (int)k;
        }
    }
    void discard(uint64_t n) {  // whole blocks are twisted, never tempered
        while (n) {
            if (pos_ == kN) twist();
            const uint64_t k = std::min<uint64_t>(n, (uint64_t)(kN - pos_));
            pos_ += (int)k;
            n -= k;
        }
    }
};

// torch.rand float32 from one 32-bit MT19937 draw.
inline float u24(uint32_t r) { return (float)(r & 0xFFFFFFu) * 0x1.0p-24f; }

// Formations [f0, f0 + cnt) from their draws u[cnt * (2N + 2)] (simulate.py:133-143: per
// formation N (x, y) pairs, then the goal pair), with each value's staging tag for generation
// `gen` when `at` is given (fenv_internal.h), taken while the bits are in registers.
FENV_HOST_CLONES void formations_from_draws(const uint32_t *u, int64_t f0, int64_t cnt, int64_t N,
                                            float *px, float *py, float *gx, float *gy,
                                            uint32_t gen, uint32_t *at, uint32_t *gt) {
    const int64_t per = 2 * N + 2;
    for (int64_t i = 0; i < cnt; ++i) {
        const uint32_t *r = u + i * per;
        const int64_t f = f0 + i;
        for (int64_t j = 0; j < N; ++j) {
            const int64_t a = f * N + j;
            const float x = u24(r[2 * j]) * 400.0f, y = u24(r[2 * j + 1]) * 100.0f;
            px[a] = x;
            py[a] = y;
            if (at) {
                uint32_t bx, by;
                std::memcpy(&bx, &x, 4);
                std::memcpy(&by, &y, 4);
                at[a] = fenvk::stage_tag_agent(gen, a, bx, by);
            }
        }
        const float g0 = u24(r[2 * N]) * 280.0f + 60.0f;
        const float g1 = u24(r[2 * N + 1]) * 480.0f + 60.0f;
        gx[f] = g0;
        gy[f] = g1;
        if (gt) {
            uint32_t bx, by;
            std::memcpy(&bx, &g0, 4);
            std::memcpy(&by, &g1, 4);
            gt[f] = fenvk::stage_tag_goal(gen, f, bx, by);
        }
    }
}

// Words of the chunk buffer draw_formations needs for `count` formations of N agents.
size_t draw_scratch_words(int64_t N, int64_t count) {
    const int64_t per = 2 * N + 2;
    const int64_t chunk = std::max<int64_t>(1, 49152 / per);
    return (size_t)(std::min<int64_t>(chunk, std::max<int64_t>(count, 1)) * per);
}

// `count` formations' reset draws from the stream's current position, in chunks of ~48K draws
// (an L2-resident buffer, `u`, at least draw_scratch_words(N, count) words): a chunk's draws in
// one fill, then its formations in one pass.  Allocates nothing, so it cannot throw: the
// draw-ahead thread runs it.
// Formations [fbase, fbase + count) of the arrays px / py / gx / gy (and their tags) are drawn;
// the stream must stand at formation fbase's first draw.
void draw_formations(Mt19937 &mt, int64_t N, int64_t count, uint32_t *u, float *px, float *py,
                     float *gx, float *gy, uint32_t gen = 0, uint32_t *at = nullptr,
                     uint32_t *gt = nullptr, int64_t fbase = 0) {
    const int64_t per = 2 * N + 2;
    const int64_t chunk = std::max<int64_t>(1, 49152 / per);
    for (int64_t f0 = 0; f0 < count; f0 += chunk) {
        const int64_t cnt = std::min<int64_t>(chunk, count - f0);
        mt.fill(u, (size_t)(cnt * per));
        formations_from_draws(u, fbase + f0, cnt, N, px, py, gx, gy, gen, at, gt);
    }
}

// A shard's draw set in up to kDrawParts parts on that many host threads: part p starts from a
// copy of the stream advanced to its first formation (discard twists whole blocks without
// tempering them, ~3x cheaper per word than a draw), so a config-3 set (12.6M draws) takes a
// third of the single-thread time; the bits are the single-thread ones.  Sets under
// kDrawSplitMin draws run on one thread.
constexpr int kDrawParts = 4;
constexpr int64_t kDrawSplitMin = (int64_t)1 << 20;
int draw_parts(int64_t N, int64_t F) { return (2 * N + 2) * F >= kDrawSplitMin ? kDrawParts : 1; }

// Formations [0, F) from the stream's current position, in draw_parts(N, F) parts (chunk buffer
// of part p at bufs + p * words, words >= draw_scratch_words(N, ceil(F / parts))); leaves mt at
// formation F's first draw.  Allocates nothing; a thread that cannot be started runs its part on
// the calling thread.
void draw_formations_par(Mt19937 &mt, int64_t N, int64_t F, uint32_t *bufs, size_t words,
                         float *px, float *py, float *gx, float *gy, uint32_t gen = 0,
                         uint32_t *at = nullptr, uint32_t *gt = nullptr) {
    const uint64_t per = 2ull * (uint64_t)N + 2ull;
    const int P = draw_parts(N, F);
    auto b = [&](int p) { return F * p / P; };  // part p: formations [b(p), b(p + 1))
    auto part = [&](int p, Mt19937 &m) {
        draw_formations(m, N, b(p + 1) - b(p), bufs + (size_t)p * words, px, py, gx, gy, gen, at,
                        gt, b(p));
    };
    Mt19937 ms[kDrawParts];
    std::thread th[kDrawParts];
    for (int p = 1; p < P; ++p) {
        ms[p] = mt;
        ms[p].discard(per * (uint64_t)b(p));
        try {
            th[p] = std::thread([&part, &ms, p]() { part(p, ms[p]); });
        } catch (...) {
            part(p, ms[p]);
        }
    }
    part(0, mt);
    for (int p = 1; p < P; ++p)
        if (th[p].joinable()) th[p].join();
    if (P > 1) mt = ms[P - 1];  // the last part's stream ends at formation F
}

// Device frees the runtime refused because a stream capture was under way (a hipFree inside a
// capture is not allowed and would invalidate it): parked here, retried at the next
// fenv_create / fenv_destroy, so fenv_destroy is safe to call at any point.
struct Graveyard {
    std::mutex mu;
    std::vector<std::pair<int32_t, void *>> dev;   // (device, pointer) for hipFree
    std::vector<std::pair<int32_t, void *>> host;  // for hipHostFree
};
Graveyard &graveyard() {
    static Graveyard *g = new Graveyard();  // never destroyed: usable from atexit / finalizers
    return *g;
}
bool capture_error(hipError_t e) {
    return e == hipErrorStreamCaptureUnsupported || e == hipErrorStreamCaptureImplicit ||
           e == hipErrorStreamCaptureInvalidated || e == hipErrorCapturedEvent;
}
void free_dev(int32_t device, void *p) {
    if (!p) return;
    if (capture_error(hipFree(p))) {
        (void)hipGetLastError();
        std::lock_guard<std::mutex> lk(graveyard().mu);
        graveyard().dev.emplace_back(device, p);
    }
}
void free_host(int32_t device, void *p) {
    if (!p) return;
    if (capture_error(hipHostFree(p))) {
        (void)hipGetLastError();
        std::lock_guard<std::mutex> lk(graveyard().mu);
        graveyard().host.emplace_back(device, p);
    }
}
// Pinned staging buffers of the MT19937 reset sets are pooled per device: a destroyed env's
// buffer goes back to its device's pool and the next env on that device takes the smallest that
// fits (never one more than 4x the request), so host staging addresses are not released and
// re-mapped on every env churn.  The pool is bounded: a buffer returned while the device's pool
// already caches kPoolCap bytes is freed (hipHostFree, parked if a capture is under way).
constexpr size_t kPoolCap = (size_t)512 << 20;
struct PinnedPool {
    std::mutex mu;
    // device -> (bytes -> (host, device address))
    std::map<int32_t, std::multimap<size_t, std::pair<float *, float *>>> free;
    std::map<int32_t, size_t> cached;
};
PinnedPool &pinned_pool() {
    static PinnedPool *p = new PinnedPool();  // never destroyed: usable from atexit / finalizers
    return *p;
}
hipError_t pinned_take(int32_t device, size_t bytes, float **host, float **dev) {
    {
        std::lock_guard<std::mutex> lk(pinned_pool().mu);
        auto &fl = pinned_pool().free[device];
        auto it = fl.lower_bound(bytes);
        if (it != fl.end() && it->first <= 4 * bytes) {
            *host = it->second.first;
            *dev = it->second.second;
            pinned_pool().cached[device] -= it->first;
            fl.erase(it);
            return hipSuccess;
        }
    }
    void *h = nullptr;
    hipError_t he = hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent |
                                                 hipHostMallocPortable);
    if (he != hipSuccess) return he;
    void *d = nullptr;
    he = hipHostGetDevicePointer(&d, h, 0);
    if (he != hipSuccess) {
        (void)hipHostFree(h);
        return he;
    }
    // the pool entry records its capacity and device address in the header before the buffer
    *reinterpret_cast<size_t *>(h) = bytes;
    reinterpret_cast<void **>(h)[1] = d;
    *host = reinterpret_cast<float *>(reinterpret_cast<char *>(h) + 256);
    *dev = reinterpret_cast<float *>(reinterpret_cast<char *>(d) + 256);
    return hipSuccess;
}
void pinned_give(int32_t device, float *host, float *dev) {
    if (!host) return;
    char *base = reinterpret_cast<char *>(host) - 256;
    const size_t bytes = *reinterpret_cast<size_t *>(base);
    {
        std::lock_guard<std::mutex> lk(pinned_pool().mu);
        size_t &c = pinned_pool().cached[device];
        if (c + bytes <= kPoolCap) {
            pinned_pool().free[device].emplace(bytes, std::make_pair(host, dev));
            c += bytes;
            return;
        }
    }
    free_host(device, base);
}
// Blocks handed out by fenv_host_alloc and not yet freed (device, host address): fenv_host_free
// of anything else returns FENV_EINVAL without reading it.
std::mutex g_host_blocks_mu;
std::map<void *, int32_t> &host_blocks() {
    static auto *m = new std::map<void *, int32_t>();  // never destroyed: usable from finalizers
    return *m;
}

size_t pinned_cached(int32_t device) {
    std::lock_guard<std::mutex> lk(pinned_pool().mu);
    auto it = pinned_pool().cached.find(device);
    return it == pinned_pool().cached.end() ? 0 : it->second;
}
// Test hook of the staging (fenv_test_stage_hook): the next g_stage_n refills run in mode
// g_stage_mode (1: the copy kernel sleeps first; 2: the copy is skipped).
std::atomic<int32_t> g_stage_mode{0}, g_stage_n{0};
// Retry the parked frees (each is parked again if a capture is still under way).
void drain_graveyard() {
    std::vector<std::pair<int32_t, void *>> dev, host;
    {
        std::lock_guard<std::mutex> lk(graveyard().mu);
        dev.swap(graveyard().dev);
        host.swap(graveyard().host);
    }
    for (auto &d : dev) {
        (void)hipSetDevice(d.first);
        free_dev(d.first, d.second);
    }
    for (auto &h : host) free_host(h.first, h.second);
}

// Live handles: fenv_create registers, fenv_destroy takes out.  A pointer that is not in the set
// (destroyed already, or never created) is refused without touching its memory.
struct LiveSet {
    std::mutex mu;
    std::unordered_set<const void *> set;
};
LiveSet &live() {
    static LiveSet *l = new LiveSet();  // never destroyed: usable from atexit / finalizers
    return *l;
}
void live_add(const void *e) {
    std::lock_guard<std::mutex> lk(live().mu);
    live().set.insert(e);
}
bool live_take(const void *e) {
    std::lock_guard<std::mutex> lk(live().mu);
    return live().set.erase(e) == 1;
}

}  // namespace

struct fenv {
    int32_t device = 0;
    fenvk::Consts c{};
    int32_t D = 8;
    int32_t goal_in_obs = 1;
    uint32_t seed = 0;
    int64_t total = 0;  // formations in the whole (unsharded) batch
    int64_t A = 0;
    fenvk::DevState s{};
    // MT19937 reset sets, double-buffered: slot k of `pend` (device) and of `hpend` (pinned,
    // coherent host memory, copied by DMA on the staging stream `cs`) each hold one set,
    // px[A] py[A] gx[F] gy[F].  `rd` is the slot the next reset event reads; a refill writes the
    // other slot, so it never touches a set a queued launch may still read, and the host only
    // rewrites a host slot whose copy (two refills back) has finished.
    float *pend = nullptr;
    float *hpend = nullptr;
    float *hpend_dev = nullptr;
    uint32_t gen_next = 1;                // generation of the next set drawn (1: the ctor's)
    uint32_t slot_gen[2] = {0u, 0u};      // generation each slot holds
    uint32_t *err_host = nullptr;         // the kernels' staging error words [4] (pinned)
    uint32_t *err_dev = nullptr;          // their mapped device address
    hipEvent_t pend_ev[2] = {nullptr, nullptr};  // staging copy of slot k done
    hipEvent_t used_ev[2] = {nullptr, nullptr};  // the launch that consumed slot k is done
    bool pend_ev_recorded[2] = {false, false};
    bool used_ev_recorded[2] = {false, false};
    int rd = 1;
    float *term = nullptr;   // device: terminal (px, py, gx, gy)[A] of the latest done step
    bool term_valid = false; // last state-changing call was a step (t == 0 <=> reset by it)
    float *lv_scratch = nullptr;  // last values for GAE when the caller passes none
    float *lf = nullptr;     // device: large-formation exchange scratch (N > 1024 only)
    Mt19937 mt;              // the reference's global stream (all formations of all shards)
    int64_t t_common = 0;    // steps_since_reset shared by all formations, -1 if not uniform
    // The next set is drawn ahead, on a host thread, while the device runs the episode: at a
    // reset event the host only stages a set drawn ~1,000 steps earlier (a config-3 set is 12.6M
    // MT19937 draws, tens of ms of host time, about one episode of device time).  The thread
    // does CPU work only -- mt, the host slot `ahead_slot`, its tags -- never a HIP call, so it
    // cannot disturb a stream capture elsewhere in the process.  mt and that host slot belong
    // to the thread until it is joined (join_ahead), and nothing else touches mt.
    std::thread ahead;
    // draw_set's chunk buffer, sized at fenv_create: the thread's body allocates nothing, so no
    // std::bad_alloc can escape it (an exception leaving a std::thread calls std::terminate)
    std::vector<uint32_t> draw_buf;  // draw_parts(N, F) chunk buffers, back to back
    size_t draw_buf_words = 0;        // words per part
    // the staging copies run on this stream (SDMA, hipMemcpyAsync from the pinned host slot), so
    // a refill overlaps the episode's launches instead of queueing 1.4 ms of PCIe-bound copy in
    // front of them; consumers wait for pend_ev, the copy waits for the slot's previous reader
    hipStream_t cs = nullptr;
    int ahead_slot = -1;     // host slot the thread is drawing into (-1: none)
    uint32_t ahead_gen = 0;  // the generation it is drawing

    size_t pend_floats() const { return (size_t)fenvk::stage_floats(A, c.F); }
    size_t pend_stride() const { return (pend_floats() + 63) & ~(size_t)63; }  // 256-B slots
    fenvk::DevPending pending() const {
        return fenvk::DevPending{pend ? pend + (size_t)rd * pend_stride() : nullptr,
                                 reinterpret_cast<float4 *>(term), lf, err_dev, slot_gen[rd]};
    }
    // The constants a rollout launch runs with.  In MT19937 mode the formations move in lock-step
    // and the host knows which launch holds the reset event (rollout_impl's `event`); a launch
    // without one takes no reset branch, so it runs the Philox instantiation of the same kernel
    // -- identical code outside that branch, where the MT19937 instantiation's staged-set reads
    // cost the config-3 launch ~4 % through register allocation (467.9 vs 449.4 us,
    // profiles/r5_mt_mode/).  Padding lanes that reach a phantom done draw into registers only.
    fenvk::Consts launch_consts(bool event) const {
        fenvk::Consts k = c;
        if (k.reset_mode == FENV_RESET_MT19937 && !event) k.reset_mode = FENV_RESET_PHILOX;
        return k;
    }

    // A staged set failed the kernels' tag check in an earlier launch (DevPending): the state
    // may hold wrong draws, so every later call on the handle fails.
    int stage_check() const {
        if (!err_host || err_host[0] == 0u) return FENV_OK;
        static const char *kinds[] = {"", "the slot's previous set (two refills back)",
                                      "the other slot's set", "neither set (corrupt)"};
        const uint32_t k = err_host[0] < 4u ? err_host[0] : 3u;
        return fail(FENV_ESTATE, std::string("MT19937 reset: a kernel read a staged draw set "
                                             "that failed its tag check (generation ") +
                                     std::to_string(err_host[1]) + ", formation " +
                                     std::to_string(err_host[2]) + "): it read " + kinds[k] +
                                     "; the env state is not the reference's -- recreate it");
    }

    // A launch that may read the staged set waits (on the device) for its refill, which may have
    // been issued on another stream.
    int wait_pending(hipStream_t st) {
        if (c.reset_mode == FENV_RESET_MT19937 && pend_ev_recorded[rd])
            FENV_HIP(hipStreamWaitEvent(st, pend_ev[rd], 0));
        return FENV_OK;
    }

    // Draw the global stream's next reset set, keep this shard's part in host slot w with its
    // tags (generation gen).  CPU only: runs on the calling thread or on `ahead`.
    void draw_set(int w, uint32_t gen) {
        const size_t off = (size_t)w * pend_stride();
        const uint64_t per = 2ull * (uint64_t)c.N + 2ull;
        mt.discard(per * (uint64_t)c.f0);
        float *hp = hpend + off;
        uint32_t *at = reinterpret_cast<uint32_t *>(hp + 2 * A + 2 * c.F);
        draw_formations_par(mt, c.N, c.F, draw_buf.data(), draw_buf_words, hp, hp + A, hp + 2 * A,
                            hp + 2 * A + c.F, gen, at, at + A);
        mt.discard(per * (uint64_t)(total - c.f0 - c.F));
    }

    // Wait for the draw-ahead thread (if any); afterwards mt and both host slots are the
    // caller's again.
    void join_ahead() {
        if (ahead.joinable()) ahead.join();
    }

    // Called right after the launch that consumed slot rd was queued on `st`: stage the global
    // stream's next reset set into the other slot (drawn ahead, or now if no draw is ahead),
    // then start drawing the set after it into the host slot just consumed.
    int gen_pending(hipStream_t st) {
        if (c.reset_mode != FENV_RESET_MT19937) return FENV_OK;
        const int w = rd ^ 1;
        if (pend_ev_recorded[rd]) {  // slot rd now has a queued reader on st
            FENV_HIP(hipEventRecord(used_ev[rd], st));
            used_ev_recorded[rd] = true;
        }
        uint32_t gen;
        if (ahead_slot == w) {
            join_ahead();
            gen = ahead_gen;
        } else {
            join_ahead();
            if (pend_ev_recorded[w]) FENV_HIP(hipEventSynchronize(pend_ev[w]));  // host slot free
            gen = gen_next++;
            draw_set(w, gen);
        }
        ahead_slot = -1;
        const size_t off = (size_t)w * pend_stride();
        // the copy runs on the handle's staging stream, after the slot's previous reader (the
        // launch that consumed it, on whatever stream)
        if (used_ev_recorded[w]) FENV_HIP(hipStreamWaitEvent(cs, used_ev[w], 0));
        int32_t mode = 0;
        if (g_stage_n.load() > 0 && g_stage_n.fetch_sub(1) > 0) mode = g_stage_mode.load();
        if (mode == 1)  // test hook: the copy starts ~0.35 ms late (a sleeping kernel ahead of it)
            FENV_HIP(fenvk::launch_stage_copy(pend + off, hpend_dev + off, 0, 100, cs));
        if (mode != 2)
            FENV_HIP(hipMemcpyAsync(pend + off, hpend + off, pend_floats() * sizeof(float),
                                    hipMemcpyHostToDevice, cs));
        slot_gen[w] = gen;
        FENV_HIP(hipEventRecord(pend_ev[w], cs));
        pend_ev_recorded[w] = true;
        rd = w;
        // draw ahead into host slot w ^ 1 once its own copy (queued at the previous refill) has
        // read it: in steady state that copy finished an episode ago
        const int nx = w ^ 1;
        if (pend_ev_recorded[nx]) FENV_HIP(hipEventSynchronize(pend_ev[nx]));
        try {
            // draw_set allocates nothing (draw_buf is sized at fenv_create): the body cannot throw
            ahead = std::thread([this, nx, g = gen_next]() { draw_set(nx, g); });
            ahead_slot = nx;
            ahead_gen = gen_next++;
        } catch (...) {  // no thread to be had: the next refill draws on the caller's thread
            ahead_slot = -1;
        }
        return FENV_OK;
    }

    // Apply a reset to every formation (pending set or Philox) and optionally write obs.
    int apply_reset(float *obs, hipStream_t st) {
        int rc = wait_pending(st);
        if (rc) return rc;
        FENV_HIP(fenvk::launch_reset_observe(c, s, pending(), D, true, obs, st));
        t_common = 0;
        term_valid = false;
        return gen_pending(st);
    }

    void advance_t(int64_t T) {
        if (t_common < 0) return;
        for (int64_t k = 0; k < T; ++k) t_common = (t_common > c.max_steps) ? 0 : t_common + 1;
    }
};

extern "C" {

const char *fenv_last_error(void) { return g_err.c_str(); }

int fenv_abi_version(void) { return FENV_ABI_VERSION; }

float fenv_desired_neighbor_dist(int32_t num_agents) {
    // simulate.py:26 in float64 (numpy), rounded to fp32 where it meets the fp32 tensor.
    return (float)(2.0 * 60.0 * std::sin(M_PI / (double)num_agents));
}

int fenv_create(fenv_t **out, int32_t device, int64_t num_formation, int32_t num_agents,
                int32_t goal_in_obs, double share_reward_ratio, int32_t max_steps, uint32_t seed,
                int32_t reset_mode, int64_t first_formation, int64_t total_formations) {
    if (!out) return fail(FENV_EINVAL, "fenv_create: out is NULL");
    *out = nullptr;
    if (num_formation < 1) return fail(FENV_EINVAL, "num_formation must be >= 1");
    if (num_agents < 1 || num_agents > FENV_MAX_AGENTS)
        return fail(FENV_EINVAL, "num_agents_per_formation must be in [1, FENV_MAX_AGENTS]");
    if (!(share_reward_ratio >= 0.0 && share_reward_ratio <= 0.5))
        return fail(FENV_EINVAL, "share_reward_ratio must be in [0, 0.5] (simulate.py:28)");
    if (max_steps < 0) return fail(FENV_EINVAL, "max_steps must be >= 0");
    if (reset_mode != FENV_RESET_MT19937 && reset_mode != FENV_RESET_PHILOX)
        return fail(FENV_EINVAL, "reset_mode must be FENV_RESET_MT19937 or FENV_RESET_PHILOX");
    if (total_formations == 0) total_formations = num_formation;
    if (first_formation < 0 || first_formation + num_formation > total_formations)
        return fail(FENV_EINVAL, "shard [first, first+num_formation) outside total_formations");
    if (num_formation * (int64_t)num_agents > (int64_t)1 << 40)
        return fail(FENV_EINVAL, "too many agents");

    int ndev = 0;
    FENV_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(FENV_EINVAL, "device index out of range");
    int prev_dev = -1;
    FENV_HIP(hipGetDevice(&prev_dev));
    drain_graveyard();
    FENV_HIP(hipSetDevice(device));

    fenv *e = new (std::nothrow) fenv();
    if (!e) return fail(FENV_ENOMEM, "fenv_create: out of host memory");
    live_add(e);
    e->device = device;
    e->goal_in_obs = goal_in_obs ? 1 : 0;
    e->D = goal_in_obs ? 8 : 6;  // vectorized_env.py:28-31
    e->seed = seed;
    e->total = total_formations;
    e->A = num_formation * num_agents;
    fenvk::Consts &c = e->c;
    c.F = num_formation;
    c.f0 = first_formation;
    c.N = num_agents;
    c.fpw = num_agents <= 64 ? 64 / num_agents : 1;
    c.max_steps = max_steps;
    c.reset_mode = reset_mode;
    c.c_self = (float)(1.0 - 2.0 * share_reward_ratio);
    c.c_nb = (float)share_reward_ratio;
    c.d_nb = fenv_desired_neighbor_dist(num_agents);
    c.key0 = seed;
    c.key1 = 0x5EEDF00Du;
    e->mt.seed(seed);  // == torch.manual_seed(seed) -> init_genrand(seed)

    auto cleanup = [&](int code) {
        fenv_destroy(e);
        if (prev_dev >= 0) (void)hipSetDevice(prev_dev);
        return code;
    };
    const size_t A = (size_t)e->A, F = (size_t)c.F;
    hipError_t he = hipSuccess;
    char *state = nullptr;
    const size_t bytes = A * 8 + F * 16;
    he = hipMalloc(&state, bytes);
    if (he != hipSuccess) return cleanup(fail(FENV_ENOMEM, "hipMalloc(state) failed"));
    e->s.px = reinterpret_cast<float *>(state);
    e->s.py = e->s.px + A;
    e->s.gx = e->s.py + A;
    e->s.gy = e->s.gx + F;
    e->s.t = reinterpret_cast<int32_t *>(e->s.gy + F);
    e->s.ep = reinterpret_cast<uint32_t *>(e->s.t + F);
    he = hipMemset(state, 0, bytes);
    if (he != hipSuccess) return cleanup(fail(FENV_EHIP, "hipMemset(state) failed"));
    he = hipMalloc(&e->term, 4 * A * sizeof(float));
    if (he != hipSuccess) return cleanup(fail(FENV_ENOMEM, "hipMalloc(terminal state) failed"));
    he = hipMemset(e->term, 0, 4 * A * sizeof(float));
    if (he != hipSuccess) return cleanup(fail(FENV_EHIP, "hipMemset(terminal state) failed"));
    if (fenvk::large_path(num_agents)) {
        he = hipMalloc(&e->lf, fenvk::kLargeScratchPerAgent * A * sizeof(float));
        if (he != hipSuccess) return cleanup(fail(FENV_ENOMEM, "hipMalloc(exchange scratch) failed"));
    }
    if (reset_mode == FENV_RESET_MT19937) {
        const size_t pb = 2 * e->pend_stride() * sizeof(float);
        he = hipMalloc(&e->pend, pb);
        if (he != hipSuccess) return cleanup(fail(FENV_ENOMEM, "hipMalloc(pending) failed"));
        he = pinned_take(device, pb + 256, &e->hpend, &e->hpend_dev);
        if (he != hipSuccess) return cleanup(fail(FENV_ENOMEM, "hipHostMalloc(pending) failed"));
        he = hipHostMalloc(reinterpret_cast<void **>(&e->err_host), 64,
                           hipHostMallocMapped | hipHostMallocCoherent);
        if (he == hipSuccess) {
            std::memset(e->err_host, 0, 64);
            he = hipHostGetDevicePointer(reinterpret_cast<void **>(&e->err_dev), e->err_host, 0);
        }
        if (he != hipSuccess) return cleanup(fail(FENV_ENOMEM, "hipHostMalloc(error words) failed"));
        for (int k = 0; k < 2; ++k) {
            he = hipEventCreateWithFlags(&e->pend_ev[k], hipEventDisableTiming);
            if (he == hipSuccess) he = hipEventCreateWithFlags(&e->used_ev[k], hipEventDisableTiming);
            if (he != hipSuccess) return cleanup(fail(FENV_EHIP, "hipEventCreate failed"));
        }
        he = hipStreamCreateWithFlags(&e->cs, hipStreamNonBlocking);
        if (he != hipSuccess) return cleanup(fail(FENV_EHIP, "hipStreamCreate(staging) failed"));
        try {
            const int P = draw_parts(num_agents, num_formation);
            e->draw_buf_words = draw_scratch_words(num_agents, (num_formation + P - 1) / P);
            e->draw_buf.resize(e->draw_buf_words * (size_t)P);
        } catch (const std::bad_alloc &) {
            return cleanup(fail(FENV_ENOMEM, "draw buffer allocation failed"));
        }
    }
    // FormationEnv ctor: every FormationSimulator.__init__ calls reset() (simulate.py:61).
    int rc = e->gen_pending(nullptr);
    if (rc) return cleanup(rc);
    rc = e->apply_reset(nullptr, nullptr);
    if (rc) return cleanup(rc);
    he = hipStreamSynchronize(nullptr);
    if (he != hipSuccess) return cleanup(fail(FENV_EHIP, hipGetErrorString(he)));
    *out = e;
    if (prev_dev >= 0) (void)hipSetDevice(prev_dev);
    return FENV_OK;
}

// Process exit with envs never destroyed: a draw-ahead thread may still be writing its host
// slot while the HIP runtime tears down the pinned allocations.  This library's destructor runs
// before the runtime's (it depends on it) and joins every live handle's thread first.
__attribute__((destructor)) static void join_draws_at_exit() {
    std::lock_guard<std::mutex> lk(live().mu);
    for (const void *h : live().set) const_cast<fenv *>(static_cast<const fenv *>(h))->join_ahead();
}

int fenv_destroy(fenv_t *e) {
    if (!e) return FENV_OK;
    if (!live_take(e)) return fail(FENV_EINVAL, "fenv_destroy: not a live handle (destroyed twice?)");
    e->join_ahead();  // the draw-ahead thread writes the host slots freed below
    // Safe at any point: the caller's current device is restored; the handle's own staging copy
    // is waited for (hipFree then waits for the device's kernels); a free the runtime refuses
    // during a stream capture is parked and retried later instead of failing the capture.
    int prev = -1;
    const bool have_prev = hipGetDevice(&prev) == hipSuccess;
    (void)hipSetDevice(e->device);
    drain_graveyard();
    for (int k = 0; k < 2; ++k)
        if (e->pend_ev_recorded[k]) (void)hipEventSynchronize(e->pend_ev[k]);
    if (e->cs) {
        (void)hipStreamSynchronize(e->cs);
        (void)hipStreamDestroy(e->cs);
    }
    free_dev(e->device, e->s.px);
    free_dev(e->device, e->pend);
    pinned_give(e->device, e->hpend, e->hpend_dev);
    free_host(e->device, e->err_host);
    for (int k = 0; k < 2; ++k) {
        if (e->pend_ev[k]) (void)hipEventDestroy(e->pend_ev[k]);
        if (e->used_ev[k]) (void)hipEventDestroy(e->used_ev[k]);
    }
    free_dev(e->device, e->lv_scratch);
    free_dev(e->device, e->term);
    free_dev(e->device, e->lf);
    delete e;
    (void)hipGetLastError();  // leave no stale error for the caller's next error check
    if (have_prev && prev >= 0) (void)hipSetDevice(prev);
    return FENV_OK;
}

int fenv_info(const fenv_t *e, int64_t *o) {
    if (!e || !o) return fail(FENV_EINVAL, "fenv_info: NULL argument");
    o[0] = e->c.F;
    o[1] = e->c.N;
    o[2] = e->D;
    o[3] = e->A;
    o[4] = e->t_common;
    o[5] = e->c.reset_mode;
    o[6] = e->c.f0;
    o[7] = e->total;
    return FENV_OK;
}

int fenv_status(const fenv_t *e) {
    if (!e) return fail(FENV_EINVAL, "fenv_status: NULL handle");
    return e->stage_check();
}

void fenv_test_stage_hook(int32_t mode, int32_t n_refills) {
    g_stage_mode.store(mode);
    g_stage_n.store(n_refills > 0 ? n_refills : 0);
}

int64_t fenv_pinned_pool_bytes(int32_t device) { return (int64_t)pinned_cached(device); }

int fenv_host_alloc(int32_t device, int64_t bytes, void **host, void **dev) {
    if (!host || !dev || bytes < 0) return fail(FENV_EINVAL, "fenv_host_alloc: bad arguments");
    int count = 0;
    FENV_HIP(hipGetDeviceCount(&count));
    if (device < 0 || device >= count) return fail(FENV_EINVAL, "fenv_host_alloc: no such device");
    drain_graveyard();
    float *h = nullptr, *d = nullptr;
    // the pool's 256-B header precedes the block; blocks are whole 256-B units
    const size_t want = ((size_t)bytes + 255) / 256 * 256 + 256;
    if (pinned_take(device, want, &h, &d) != hipSuccess) {
        (void)hipGetLastError();
        return fail(FENV_ENOMEM, "fenv_host_alloc: hipHostMalloc failed");
    }
    {
        std::lock_guard<std::mutex> lk(g_host_blocks_mu);
        host_blocks()[h] = device;
    }
    *host = h;
    *dev = d;
    return FENV_OK;
}

int fenv_host_free(int32_t device, void *host) {
    if (!host) return FENV_OK;
    {
        std::lock_guard<std::mutex> lk(g_host_blocks_mu);
        auto it = host_blocks().find(host);
        if (it == host_blocks().end() || it->second != device)
            return fail(FENV_EINVAL, "fenv_host_free: not a live fenv_host_alloc block of this device");
        host_blocks().erase(it);
    }
    void *d = reinterpret_cast<void **>(static_cast<char *>(host) - 256)[1];
    pinned_give(device, static_cast<float *>(host),
                reinterpret_cast<float *>(static_cast<char *>(d) + 256));
    return FENV_OK;
}

int fenv_debug_staging(fenv_t *e, int32_t which, float *out_host, int64_t *info_host) {
    if (!e || !info_host) return fail(FENV_EINVAL, "fenv_debug_staging: NULL argument");
    e->join_ahead();
    info_host[0] = e->rd;
    info_host[1] = e->slot_gen[0];
    info_host[2] = e->slot_gen[1];
    info_host[3] = (int64_t)e->pend_floats();
    info_host[4] = e->err_host ? e->err_host[0] : 0;
    info_host[5] = e->err_host ? e->err_host[1] : 0;
    info_host[6] = e->err_host ? e->err_host[2] : 0;
    info_host[7] = e->gen_next;
    info_host[8] = (int64_t)reinterpret_cast<uintptr_t>(e->term);
    info_host[9] = (int64_t)reinterpret_cast<uintptr_t>(e->pend);
    if (out_host && which == 4) {  // the terminal-state records (px, py, gx, gy)[A]
        FENV_HIP(hipSetDevice(e->device));
        FENV_HIP(hipDeviceSynchronize());
        FENV_HIP(hipMemcpy(out_host, e->term, (size_t)e->A * 16, hipMemcpyDeviceToHost));
        return FENV_OK;
    }
    if (!out_host || !e->pend || which < 0 || which > 3) return FENV_OK;
    FENV_HIP(hipSetDevice(e->device));
    const size_t off = (size_t)(which & 1) * e->pend_stride();
    if (which < 2)
        FENV_HIP(hipMemcpy(out_host, e->pend + off, e->pend_floats() * 4, hipMemcpyDeviceToHost));
    else
        std::memcpy(out_host, e->hpend + off, e->pend_floats() * 4);
    return FENV_OK;
}

int64_t fenv_partial_count(const fenv_t *e) { return e ? fenvk::rollout_group_count(e->c) : -1; }

const char *fenv_rollout_kernel(const fenv_t *e, int32_t T) {
    return e ? fenvk::rollout_kernel_name(e->c, T) : "";
}

int fenv_reset(fenv_t *e, float *obs, void *stream) {
    if (!e) return fail(FENV_EINVAL, "fenv_reset: NULL handle");
    if (int rc = e->stage_check()) return rc;
    FENV_HIP(hipSetDevice(e->device));
    return e->apply_reset(obs, as_stream(stream));
}

int fenv_observe(fenv_t *e, float *obs, void *stream) {
    if (!e || !obs) return fail(FENV_EINVAL, "fenv_observe: NULL argument");
    if (int rc = e->stage_check()) return rc;
    FENV_HIP(hipSetDevice(e->device));
    FENV_HIP(fenvk::launch_reset_observe(e->c, e->s, e->pending(), e->D, false, obs,
                                        as_stream(stream)));
    return FENV_OK;
}

// fenv_rollout / fenv_rollout_random: T fused steps, split at MT19937 reset events.  gen = NULL:
// actions from `act`; else generated in the kernel (gen->offset / gen->out advance per launch).
static int rollout_impl(fenv_t *e, int32_t T, const float *act, const fenvk::ActGen *gen,
                        float *obs, float *rew, uint8_t *done, float *partial, void *stream) {
    if (int rc = e->stage_check()) return rc;
    FENV_HIP(hipSetDevice(e->device));
    hipStream_t st = as_stream(stream);
    const int64_t A = e->A, D = e->D;
    int64_t k0 = 0;
    if (T > 0) {
        int rc = e->wait_pending(st);
        if (rc) return rc;
        e->term_valid = true;
    }
    const bool nt = fenvk::rollout_nt(e->c, T);
    const int64_t chunk = fenvk::rollout_launch_steps(e->c, T);
    while (k0 < T) {
        int64_t L = std::min<int64_t>(T - k0, chunk);
        bool event = false;
        if (e->c.reset_mode == FENV_RESET_MT19937) {
            if (e->t_common < 0)
                return fail(FENV_ESTATE, "MT19937 reset mode needs formations in lock-step");
            // first local step whose pre-step t exceeds max_steps (simulate.py:231)
            const int64_t je = std::max<int64_t>(0, (int64_t)e->c.max_steps + 1 - e->t_common);
            if (je < L) {
                L = je + 1;  // this launch ends with the reset event
                event = true;
            }
        }
        fenvk::ActGen g{};
        if (gen) {
            g = *gen;
            g.offset += (uint64_t)k0;
            if (g.out) g.out += k0 * A * 2;
        }
        FENV_HIP(fenvk::launch_rollout(
            e->launch_consts(event), e->s, e->pending(), (int32_t)L, (int32_t)D, act ? act + k0 * A * 2 : nullptr,
            obs ? obs + k0 * A * D : nullptr, rew ? rew + k0 * A : nullptr,
            done ? done + k0 * A : nullptr, partial, k0 > 0, nt, st, gen ? &g : nullptr));
        e->advance_t(L);
        if (event) {
            int rc = e->gen_pending(st);
            // the call's next launch reads the set just staged: its copy runs on the staging
            // stream, so the launch stream waits for it (round 5's staging A/B caught the missing
            // wait with the delayed-copy test hook; profiles/r5_mt_mode/README.txt)
            if (!rc && k0 + L < T) rc = e->wait_pending(st);
            if (rc) return rc;
        }
        k0 += L;
    }
    return FENV_OK;
}

int fenv_rollout(fenv_t *e, int32_t T, const float *act, float *obs, float *rew, uint8_t *done,
                 float *partial, void *stream) {
    if (!e) return fail(FENV_EINVAL, "fenv_rollout: NULL handle");
    if (T < 0) return fail(FENV_EINVAL, "fenv_rollout: T must be >= 0");
    if (!act && T > 0) return fail(FENV_EINVAL, "fenv_rollout: act is NULL");
    return rollout_impl(e, T, act, nullptr, obs, rew, done, partial, stream);
}

int fenv_rollout_random(fenv_t *e, int32_t T, uint64_t act_seed, uint64_t step_offset,
                        float *act_out, float *obs, float *rew, uint8_t *done, float *partial,
                        void *stream) {
    if (!e) return fail(FENV_EINVAL, "fenv_rollout_random: NULL handle");
    if (T < 0) return fail(FENV_EINVAL, "fenv_rollout_random: T must be >= 0");
    fenvk::ActGen g{};
    g.k0 = (uint32_t)act_seed;
    g.k1 = (uint32_t)(act_seed >> 32);
    g.offset = step_offset;
    g.out = act_out;
    return rollout_impl(e, T, nullptr, &g, obs, rew, done, partial, stream);
}

int fenv_step(fenv_t *e, const float *act, float *obs, float *rew, uint8_t *done, void *stream) {
    return fenv_rollout(e, 1, act, obs, rew, done, nullptr, stream);
}

int fenv_reduce_partials(const float *partial, int64_t count, double *out, void *stream) {
    if (!partial || !out || count < 0) return fail(FENV_EINVAL, "fenv_reduce_partials: bad args");
    FENV_HIP(fenvk::launch_reduce_partials(partial, count, out, as_stream(stream)));
    return FENV_OK;
}

int fenv_stream_gate(const uint32_t *flag, uint32_t value, int64_t timeout_us, uint32_t *status,
                     void *stream) {
    if (!flag || timeout_us <= 0 || timeout_us > 60000000)
        return fail(FENV_EINVAL, "fenv_stream_gate: NULL flag or timeout_us not in (0, 60 s]");
    int dev = 0, khz = 0;
    FENV_HIP(hipGetDevice(&dev));
    FENV_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    if (khz <= 0) return fail(FENV_EHIP, "fenv_stream_gate: no wall-clock rate");
    const uint64_t ticks = (uint64_t)timeout_us * (uint64_t)khz / 1000u;
    FENV_HIP(fenvk::launch_stream_gate(flag, value, ticks, (uint32_t)khz, status,
                                       as_stream(stream)));
    return FENV_OK;
}

int fenv_metrics(fenv_t *e, const float *rew, float *out, double *sums, void *stream) {
    if (!e || !out) return fail(FENV_EINVAL, "fenv_metrics: NULL argument");
    if (int rc = e->stage_check()) return rc;
    FENV_HIP(hipSetDevice(e->device));
    FENV_HIP(fenvk::launch_metrics(e->c, e->s, e->pending(), e->term_valid, rew, out, sums,
                                   as_stream(stream)));
    return FENV_OK;
}

int fenv_get_state(fenv_t *e, float *px, float *py, float *gx, float *gy, int32_t *t,
                   void *stream) {
    if (!e) return fail(FENV_EINVAL, "fenv_get_state: NULL handle");
    if (int rc = e->stage_check()) return rc;
    FENV_HIP(hipSetDevice(e->device));
    hipStream_t st = as_stream(stream);
    const size_t A = (size_t)e->A, F = (size_t)e->c.F;
    if (px) FENV_HIP(hipMemcpyAsync(px, e->s.px, A * 4, hipMemcpyDeviceToDevice, st));
    if (py) FENV_HIP(hipMemcpyAsync(py, e->s.py, A * 4, hipMemcpyDeviceToDevice, st));
    if (gx) FENV_HIP(hipMemcpyAsync(gx, e->s.gx, F * 4, hipMemcpyDeviceToDevice, st));
    if (gy) FENV_HIP(hipMemcpyAsync(gy, e->s.gy, F * 4, hipMemcpyDeviceToDevice, st));
    if (t) FENV_HIP(hipMemcpyAsync(t, e->s.t, F * 4, hipMemcpyDeviceToDevice, st));
    return FENV_OK;
}

int fenv_get_state_range(fenv_t *e, int64_t first, int64_t count, float *px, float *py,
                         float *gx, float *gy, int32_t *t, void *stream) {
    if (!e) return fail(FENV_EINVAL, "fenv_get_state_range: NULL handle");
    if (int rc = e->stage_check()) return rc;
    if (first < 0 || count < 1 || first + count > e->c.F)
        return fail(FENV_EINVAL, "fenv_get_state_range: formations outside the handle's shard");
    FENV_HIP(hipSetDevice(e->device));
    hipStream_t st = as_stream(stream);
    const size_t a0 = (size_t)first * e->c.N, na = (size_t)count * e->c.N, nf = (size_t)count;
    if (px) FENV_HIP(hipMemcpyAsync(px, e->s.px + a0, na * 4, hipMemcpyDeviceToDevice, st));
    if (py) FENV_HIP(hipMemcpyAsync(py, e->s.py + a0, na * 4, hipMemcpyDeviceToDevice, st));
    if (gx) FENV_HIP(hipMemcpyAsync(gx, e->s.gx + first, nf * 4, hipMemcpyDeviceToDevice, st));
    if (gy) FENV_HIP(hipMemcpyAsync(gy, e->s.gy + first, nf * 4, hipMemcpyDeviceToDevice, st));
    if (t) FENV_HIP(hipMemcpyAsync(t, e->s.t + first, nf * 4, hipMemcpyDeviceToDevice, st));
    return FENV_OK;
}

int fenv_metrics_range(fenv_t *e, int64_t first, int64_t count, const float *rew, float *out,
                       double *sums, void *stream) {
    if (!e || !out) return fail(FENV_EINVAL, "fenv_metrics_range: NULL argument");
    if (int rc = e->stage_check()) return rc;
    if (first < 0 || count < 1 || first + count > e->c.F)
        return fail(FENV_EINVAL, "fenv_metrics_range: formations outside the handle's shard");
    FENV_HIP(hipSetDevice(e->device));
    // the metrics kernels over a sub-shard: the same kernels on views of the state arrays
    fenvk::Consts c = e->c;
    c.F = count;
    c.f0 = e->c.f0 + first;
    const int64_t a0 = first * (int64_t)e->c.N;
    fenvk::DevState s{e->s.px + a0, e->s.py + a0, e->s.gx + first, e->s.gy + first,
                      e->s.t + first, e->s.ep + first};
    fenvk::DevPending p = e->pending();
    p.term += a0;
    FENV_HIP(fenvk::launch_metrics(c, s, p, e->term_valid, rew, out, sums, as_stream(stream)));
    return FENV_OK;
}

int fenv_set_state(fenv_t *e, const float *px, const float *py, const float *gx, const float *gy,
                   const int32_t *t, void *stream) {
    if (!e || !px || !py || !gx || !gy || !t) return fail(FENV_EINVAL, "fenv_set_state: NULL");
    if (int rc = e->stage_check()) return rc;
    FENV_HIP(hipSetDevice(e->device));
    hipStream_t st = as_stream(stream);
    const size_t A = (size_t)e->A, F = (size_t)e->c.F;
    std::vector<int32_t> ht(F);
    FENV_HIP(hipMemcpyAsync(ht.data(), t, F * 4, hipMemcpyDeviceToHost, st));
    FENV_HIP(hipStreamSynchronize(st));
    int64_t tc = ht[0];
    for (size_t f = 0; f < F; ++f) {
        if (ht[f] < 0) return fail(FENV_EINVAL, "fenv_set_state: negative steps_since_reset");
        if (ht[f] != ht[0]) tc = -1;
    }
    if (tc < 0 && e->c.reset_mode == FENV_RESET_MT19937)
        return fail(FENV_EINVAL,
                    "fenv_set_state: MT19937 reset mode replays the reference's global stream and "
                    "needs every formation at the same steps_since_reset; use FENV_RESET_PHILOX");
    FENV_HIP(hipMemcpyAsync(e->s.px, px, A * 4, hipMemcpyDeviceToDevice, st));
    FENV_HIP(hipMemcpyAsync(e->s.py, py, A * 4, hipMemcpyDeviceToDevice, st));
    FENV_HIP(hipMemcpyAsync(e->s.gx, gx, F * 4, hipMemcpyDeviceToDevice, st));
    FENV_HIP(hipMemcpyAsync(e->s.gy, gy, F * 4, hipMemcpyDeviceToDevice, st));
    FENV_HIP(hipMemcpyAsync(e->s.t, t, F * 4, hipMemcpyDeviceToDevice, st));
    e->t_common = tc;
    e->term_valid = false;
    return FENV_OK;
}

int fenv_host_reset_draws(uint32_t seed, int64_t skip_sets, int64_t total, int64_t first,
                          int64_t count, int32_t num_agents, float *px, float *py, float *gx,
                          float *gy) {
    if (num_agents < 1 || total < 0 || first < 0 || count < 0 || first + count > total ||
        skip_sets < 0 || (count > 0 && (!px || !py || !gx || !gy)))
        return fail(FENV_EINVAL, "fenv_host_reset_draws: bad arguments");
    std::vector<uint32_t> u;
    const int P = draw_parts(num_agents, count);
    const size_t words = draw_scratch_words(num_agents, (count + P - 1) / P);
    try {
        u.resize(words * (size_t)P);
    } catch (const std::bad_alloc &) {
        return fail(FENV_ENOMEM, "fenv_host_reset_draws: out of host memory");
    }
    Mt19937 mt;
    mt.seed(seed);
    const uint64_t per = 2ull * (uint64_t)num_agents + 2ull;
    mt.discard(per * ((uint64_t)skip_sets * (uint64_t)total + (uint64_t)first));
    draw_formations_par(mt, num_agents, count, u.data(), words, px, py, gx, gy);
    return FENV_OK;
}

// Diagnostic: run one of the kernels' fp32 primitives over n inputs on the device
// (op 0: x/400, 1: x/600, 2: sqrtf(x), 3: sqrtf(fmaf(y, y, x*x))).  Device pointers.
int fenv_fp_probe(int32_t op, const float *a, const float *b, float *out, int64_t n,
                  void *stream) {
    if (!a || !out || n < 0 || op < 0 || op > 3 || (op == 3 && !b))
        return fail(FENV_EINVAL, "fenv_fp_probe: bad arguments");
    FENV_HIP(fenvk::launch_fp_probe(op, a, b, out, n, as_stream(stream)));
    return FENV_OK;
}

int policy_param_count(int32_t obs_dim) {
    // 2 x (D*64 + 64 + 64*64 + 64) + (2*64 + 2) + (64 + 1) + 2 (log_std)
    return 2 * (obs_dim * 64 + 64 + 64 * 64 + 64) + 130 + 65 + 2;
}

int policy_forward(const float *params, int32_t obs_dim, const float *obs, int64_t B,
                   int64_t row0, float *mu, float *value, float *action, float *logp,
                   float *clipped, uint64_t seed, uint64_t offset, int32_t deterministic,
                   void *stream) {
    if (!params || !obs || B < 0 || row0 < 0 || (obs_dim != 6 && obs_dim != 8))
        return fail(FENV_EINVAL, "policy_forward: bad arguments (obs_dim must be 6 or 8)");
    if (B == 0) return FENV_OK;
    FENV_HIP(fenvk::launch_policy_forward(params, obs_dim, obs, B, row0, mu, value, action, logp,
                                         clipped, seed, offset, deterministic, as_stream(stream)));
    return FENV_OK;
}

int fenv_policy_rollout(fenv_t *e, const float *params, int32_t T, uint64_t seed,
                        uint64_t offset, int32_t deterministic, float gamma, float gae_lambda,
                        const fenv_rollout_bufs *bufs, void *stream) {
    if (!e || !params || !bufs) return fail(FENV_EINVAL, "fenv_policy_rollout: NULL argument");
    if (int rc = e->stage_check()) return rc;
    if (T < 1) return fail(FENV_EINVAL, "fenv_policy_rollout: T must be >= 1");
    const fenv_rollout_bufs &b = *bufs;
    if (!b.obs || !b.action || !b.value || !b.log_prob || !b.reward || !b.episode_start ||
        !b.last_done)
        return fail(FENV_EINVAL, "fenv_policy_rollout: obs, action, value, log_prob, reward, "
                                 "episode_start and last_done are required");
    if ((b.advantage == nullptr) != (b.ret == nullptr))
        return fail(FENV_EINVAL, "fenv_policy_rollout: advantage and ret go together");
    if (!fenvk::wave_path(e->c.N))
        return fail(FENV_EINVAL, "fenv_policy_rollout: num_agents must be <= 64 "
                                 "(use policy_forward + fenv_step for larger formations)");
    FENV_HIP(hipSetDevice(e->device));
    hipStream_t st = as_stream(stream);
    bool event = false;
    if (e->c.reset_mode == FENV_RESET_MT19937) {
        if (e->t_common < 0)
            return fail(FENV_ESTATE, "MT19937 reset mode needs formations in lock-step");
        const int64_t je = std::max<int64_t>(0, (int64_t)e->c.max_steps + 1 - e->t_common);
        if (je < T) {
            event = true;
            if (je + (int64_t)e->c.max_steps + 2 < T)
                return fail(FENV_EINVAL, "fenv_policy_rollout: more than one reset event in one "
                                         "launch (T > max_steps + 2) in MT19937 mode");
        }
    }
    int rc0 = e->wait_pending(st);
    if (rc0) return rc0;
    e->term_valid = true;
    const bool gae = b.advantage != nullptr;
    fenvk::PRArgs g{};
    g.b = b;
    g.params = params;
    g.T = T;
    g.deterministic = deterministic;
    g.seed = seed;
    g.offset = offset;
    g.gamma = gamma;
    g.lam = gae_lambda;
    if (gae && !b.last_value) {  // GAE needs the last values
        if (!e->lv_scratch) {
            hipError_t he = hipMalloc(&e->lv_scratch, (size_t)e->A * sizeof(float));
            if (he != hipSuccess) return fail(FENV_ENOMEM, "hipMalloc(last_value scratch) failed");
        }
        g.b.last_value = e->lv_scratch;
    }
    FENV_HIP(fenvk::launch_policy_rollout(e->launch_consts(event), e->s, e->pending(), e->D, g, st));
    e->advance_t(T);
    if (event) {
        int rc = e->gen_pending(st);
        if (rc) return rc;
    }
    if (gae)
        FENV_HIP(fenvk::launch_gae(b.reward, b.value, b.episode_start, g.b.last_value, b.last_done,
                                   T, e->A, gamma, gae_lambda, b.advantage, b.ret, st));
    return FENV_OK;
}

int rollout_gae(const float *rew, const float *values, const uint8_t *episode_starts,
                const float *last_values, const uint8_t *last_dones, int32_t T, int64_t A,
                float gamma, float gae_lambda, float *advantages, float *returns, void *stream) {
    if (!rew || !values || !episode_starts || !last_values || !last_dones || !advantages ||
        !returns || T < 1 || A < 1)
        return fail(FENV_EINVAL, "rollout_gae: bad arguments");
    FENV_HIP(fenvk::launch_gae(rew, values, episode_starts, last_values, last_dones, T, A, gamma,
                               gae_lambda, advantages, returns, as_stream(stream)));
    return FENV_OK;
}

static int ppo_update_impl(float *params, float *exp_avg, float *exp_avg_sq, float *step,
                           int32_t obs_dim, const float *obs, const float *actions,
                           const float *old_log_prob, const float *advantages,
                           const float *returns, int64_t n, const int64_t *perm, int32_t n_epochs,
                           int32_t batch_size, const ppo_hparams *hp, double *stats,
                           void *workspace, void *stream) {
    if (!params || !exp_avg || !exp_avg_sq || !step || !obs || !actions || !old_log_prob ||
        !advantages || !returns || !perm || !hp || !stats)
        return fail(FENV_EINVAL, "ppo_update: NULL argument");
    if (obs_dim != 6 && obs_dim != 8) return fail(FENV_EINVAL, "ppo_update: obs_dim must be 6 or 8");
    if (n < 1 || n_epochs < 0 || batch_size < 1 || batch_size > 64)
        return fail(FENV_EINVAL, "ppo_update: need n >= 1 and 1 <= batch_size <= 64");
    if (n_epochs == 0) return FENV_OK;
    FENV_HIP(fenvk::launch_ppo_update(params, exp_avg, exp_avg_sq, step, obs_dim, obs, actions,
                                      old_log_prob, advantages, returns, n, perm, n_epochs,
                                      batch_size, *hp, stats, workspace, as_stream(stream)));
    return FENV_OK;
}

int ppo_update(float *params, float *exp_avg, float *exp_avg_sq, float *step, int32_t obs_dim,
               const float *obs, const float *actions, const float *old_log_prob,
               const float *advantages, const float *returns, int64_t n, const int64_t *perm,
               int32_t n_epochs, int32_t batch_size, const ppo_hparams *hp, double *stats,
               void *stream) {
    return ppo_update_impl(params, exp_avg, exp_avg_sq, step, obs_dim, obs, actions, old_log_prob,
                           advantages, returns, n, perm, n_epochs, batch_size, hp, stats, nullptr,
                           stream);
}

int64_t ppo_workspace_bytes(void) { return (int64_t)fenvk::ppo_workspace_bytes_impl(); }

void fenv_test_ppo_inject(int32_t n_launches) { fenvk::ppo_set_inject(n_launches); }

int ppo_update_ws(float *params, float *exp_avg, float *exp_avg_sq, float *step, int32_t obs_dim,
                  const float *obs, const float *actions, const float *old_log_prob,
                  const float *advantages, const float *returns, int64_t n, const int64_t *perm,
                  int32_t n_epochs, int32_t batch_size, const ppo_hparams *hp, double *stats,
                  void *workspace, void *stream) {
    if (!workspace) return fail(FENV_EINVAL, "ppo_update_ws: NULL workspace");
    return ppo_update_impl(params, exp_avg, exp_avg_sq, step, obs_dim, obs, actions, old_log_prob,
                           advantages, returns, n, perm, n_epochs, batch_size, hp, stats,
                           workspace, stream);
}

int ppo_grad(const float *params, int32_t obs_dim, const float *obs, const float *actions,
             const float *old_log_prob, const float *advantages, const float *returns,
             const int64_t *rows, int32_t b_local, int32_t b_global, float adv_mean,
             float adv_std, int32_t adv_normalize, int32_t entropy_term, const ppo_hparams *hp,
             float *grad, double *stats, void *stream) {
    if (!params || !obs || !actions || !old_log_prob || !advantages || !returns || !hp ||
        !grad || !stats || (b_local > 0 && !rows))
        return fail(FENV_EINVAL, "ppo_grad: NULL argument");
    if (obs_dim != 6 && obs_dim != 8) return fail(FENV_EINVAL, "ppo_grad: obs_dim must be 6 or 8");
    if (b_local < 0 || b_local > 64 || b_global < 1 || b_local > b_global)
        return fail(FENV_EINVAL, "ppo_grad: need 0 <= b_local <= min(64, b_global)");
    hipStream_t st = as_stream(stream);
    if (b_local == 0) {  // no rows here: a zero gradient (+ the entropy term if this rank owns it)
        const int P = policy_param_count(obs_dim);
        FENV_HIP(hipMemsetAsync(grad, 0, (size_t)P * sizeof(float), st));
        if (entropy_term) {
            const float e[2] = {-hp->ent_coef, -hp->ent_coef};
            FENV_HIP(hipMemcpyAsync(grad + P - 2, e, sizeof(e), hipMemcpyHostToDevice, st));
            FENV_HIP(hipStreamSynchronize(st));  // e is on the host stack
        }
        return FENV_OK;
    }
    FENV_HIP(fenvk::launch_ppo_grad(params, obs_dim, obs, actions, old_log_prob, advantages,
                                    returns, rows, b_local, b_global, adv_mean, adv_std,
                                    adv_normalize, entropy_term, *hp, grad, stats, st));
    return FENV_OK;
}

int ppo_apply(float *params, float *exp_avg, float *exp_avg_sq, float *step, const float *grad,
              int32_t obs_dim, const ppo_hparams *hp, void *stream) {
    if (!params || !exp_avg || !exp_avg_sq || !step || !grad || !hp)
        return fail(FENV_EINVAL, "ppo_apply: NULL argument");
    if (obs_dim != 6 && obs_dim != 8) return fail(FENV_EINVAL, "ppo_apply: obs_dim must be 6 or 8");
    FENV_HIP(fenvk::launch_ppo_apply(params, exp_avg, exp_avg_sq, step, grad, obs_dim, *hp,
                                     as_stream(stream)));
    return FENV_OK;
}

}  // extern "C"
