// api.hip -- host orchestration and the extern "C" boundary (include/gsr.h).
//
// Forward stage order mirrors CudaRasterizer::Rasterizer::forward
// (CR/rasterizer_impl.cu:227-370); the stages themselves are this project's
// (depth pre-sort + 16-bit tile sort instead of one 64-bit sort, footprint
// culling in the blender, atomic-free backward).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <atomic>
#include <chrono>
#include <algorithm>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/gsr.h"
#include "../../include/gsr_knn.h"
#include "../../include/gsr_ssim.h"
#include "../../include/gsr_adam.h"
#include "../../include/gsr_densify.h"
#include "kernels.h"

namespace {

thread_local char g_err[1024] = "";

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

}  // namespace

namespace gsr {
// for host-only translation units (ply.cpp): set gsr_last_error()'s message, return `code`
int set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}
}  // namespace gsr

namespace {

#define HIP_TRY(expr, stage)                                                                                    \
    do {                                                                                                        \
        hipError_t _e = (expr);                                                                                 \
        if (_e != hipSuccess) return fail(GSR_ERR_HIP, "%s: %s", stage, hipGetErrorString(_e));                 \
    } while (0)

// ---- stage profiler -----------------------------------------------------------
enum Stage {
    ST_PREPROCESS = 0,
    ST_BIN_COUNT,    // K1 + K2 of binning.hip
    ST_BIN_SCATTER,  // K3
    ST_TILE_SORT,    // K4
    ST_RENDER_FWD,
    ST_RENDER_BWD,
    ST_GAUSS_REDUCE,
    ST_GAUSS_BWD,
    ST_COUNT
};
const char* kStageNames[ST_COUNT] = {"preprocess", "bin_count",  "bin_scatter",  "tile_sort",
                                     "render_fwd", "render_bwd", "gauss_reduce", "gauss_bwd"};

struct Profiler {
    unsigned mask = 0;  // bit s: record stage s
    std::mutex mu;
    struct Pending {
        int stage;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> pool;
    double total_ms[ST_COUNT] = {};
    long long calls[ST_COUNT] = {};
    hipEvent_t get() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e;
        (void)hipEventCreate(&e);
        return e;
    }
};
Profiler g_prof;
unsigned long long* g_census = nullptr;  // gsr_census_set: device counters of the census render kernels

struct StageScope {
    int stage;
    hipStream_t stream;
    hipEvent_t a = nullptr;
    StageScope(int s, hipStream_t st) : stage(s), stream(st) {
        if ((g_prof.mask >> s) & 1u) {
            std::lock_guard<std::mutex> lk(g_prof.mu);
            a = g_prof.get();
            (void)hipEventRecord(a, stream);
        }
    }
    ~StageScope() {
        if (a) {
            std::lock_guard<std::mutex> lk(g_prof.mu);
            hipEvent_t b = g_prof.get();
            (void)hipEventRecord(b, stream);
            g_prof.pending.push_back({stage, a, b});
        }
    }
};

int check_debug(int debug, hipStream_t stream, const char* stage) {
    if (!debug) return GSR_OK;
    hipError_t e = hipStreamSynchronize(stream);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) return fail(GSR_ERR_HIP, "%s: %s", stage, hipGetErrorString(e));
    return GSR_OK;
}


gsr::GeomState carve_geom(char* base, int P, uint32_t gx, uint32_t gy, size_t* total) {
    using namespace gsr;
    Carver c{base, 0};
    GeomState g{};
    g.rec = c.take<float4>((size_t)kRecRows * P);
    g.depth_key = c.take<uint32_t>(P);
    g.tiles_touched = c.take<uint32_t>(P);
    g.rect = c.take<uint2>(P);
    g.rec_start = c.take<uint32_t>(P);
    g.clamped = c.take<uint8_t>(P);
    g.status = c.take<uint32_t>(4);
    g.fwd_seg_ck = g.status + 2;
    const uint32_t tiles = gx * gy;
    const size_t cells = bin_cell_count(gx, gy);
    // the counters preprocess zeroes in one range (bin_zero_words): tile counts, cell counts, near counts,
    // the depth-mass histogram (8-byte aligned)
    g.tile_cnt = c.take<uint32_t>(bin_zero_words(tiles, cells));
    g.cell_cnt = g.tile_cnt + tiles;
    g.near_cnt = g.cell_cnt + cells;
    g.zhist = reinterpret_cast<unsigned long long*>(g.tile_cnt + ((2 * (size_t)tiles + cells + 1) & ~(size_t)1));
    g.tile_base = c.take<uint32_t>(tiles);
    const size_t chunks = bin_chunk_count(P);
    g.cell_off = c.take<uint32_t>(chunks * cells);
    g.order = c.take<uint4>(P);
    g.n_visible = c.take<uint32_t>(1);

    g.chunk_off = c.take<uint32_t>(chunks * tiles);
    g.cls_list = c.take<uint32_t>(2 * (size_t)tiles);
    g.cls_count = c.take<uint32_t>(2);
    g.chunk_total = c.take<unsigned long long>(chunks);
    g.total = c.take<unsigned long long>(1);
    g.unit_cnt = c.take<uint32_t>((size_t)kUnitLists * kUnitShards * kUnitCntStride);
    g.unit_part = c.take<uint2>((size_t)(kUnitLists - 1) * kUnitShards * unit_part_cap(tiles));
    g.tile_join = c.take<unsigned long long>(tiles);
    g.sorted_len = c.take<uint32_t>(tiles);
    g.redo_flag = c.take<uint32_t>(tiles);
    g.redo_list = c.take<uint32_t>(tiles);
    g.redo_cnt = c.take<uint32_t>(1);
    g.acc = c.take<float4>((size_t)kAccRow4 * P);
    g.touched = c.take<uint32_t>(touched_words((size_t)P));
    g.mass = c.take<uint32_t>(P);
    g.zcut = g.status + 3;
    g.sranges = c.take<uint2>(tiles);
    g.far_cur = c.take<uint32_t>(tiles);
    *total = align_up(c.off);
    return g;
}

gsr::ImageState carve_image(char* base, int W, int H, uint32_t tiles, size_t* total) {
    using namespace gsr;
    Carver c{base, 0};
    ImageState im{};
    const size_t N = (size_t)W * H;
    const size_t NT = (size_t)tiles * 256;  // tile-major pixel planes (gsr_common.h tile_px)
    (void)N;
    im.final_T = c.take<float>(NT);
    im.n_contrib = c.take<uint32_t>(NT);
    im.accum = c.take<float>(4 * NT);
    im.ranges = c.take<uint2>(tiles);
    *total = align_up(c.off);
    return im;
}

gsr::BinningState carve_binning(char* base, size_t C, size_t* total) {
    using namespace gsr;
    Carver c{base, 0};
    BinningState b{};
    b.keys = c.take<unsigned long long>(C);
    b.gid_sorted = c.take<uint32_t>(C);
    b.ckpt = c.take<float>((C / kCkStride + 1) * (size_t)kCkFloats);
    b.unit_full = c.take<uint2>(kUnitShards * unit_full_cap(C));
    b.rec_flag = c.take<uint8_t>(((C + 15) & ~(size_t)15) + 16);  // K3 / gauss_reduce use aligned 16-byte words
    *total = align_up(c.off);
    return b;
}

// Binning capacities of the _ex / _dc forwards are multiples of kCapQuantum.  Over those the
// buffer size is strictly increasing (the keys alone grow by 8 * kCapQuantum bytes a step) and
// every sub-array's length depends on C / kCkStride at most, so the size of the binning buffer
// identifies its layout: the backward recovers the capacity from the tensor's byte count, which
// survives any transport of the saved tensor (saved-tensor hooks, save_on_cpu, clone).
constexpr size_t kCapQuantum = 256;
static_assert(kCapQuantum % gsr::kCkStride == 0, "capacity quantum is a whole number of checkpoint strides");

size_t quantize_capacity(size_t c) { return (c + kCapQuantum - 1) / kCapQuantum * kCapQuantum; }

size_t binning_bytes_for(size_t C) {
    size_t b = 0;
    carve_binning(nullptr, C, &b);
    return b;
}

// Capacity the binning buffer of a forward was laid out for: the explicit value if given,
// else the multiple of kCapQuantum whose layout has exactly `bytes` bytes, else R (the exact
// layout of gsr_rasterize_forward).  Returns false if `bytes` matches no layout holding R.
bool resolve_capacity(int R, int capacity, size_t bytes, size_t* C) {
    if (capacity > 0) {
        *C = (size_t)capacity;
        return bytes == 0 || binning_bytes_for(*C) == bytes;
    }
    if (bytes == 0) {
        *C = (size_t)R;
        return true;
    }
    size_t lo = quantize_capacity((size_t)R) / kCapQuantum, hi = bytes / (8 * kCapQuantum) + 1;
    while (lo < hi) {  // first k in [lo, hi] with bytes_for(k * quantum) >= bytes
        const size_t mid = lo + (hi - lo) / 2;
        if (binning_bytes_for(mid * kCapQuantum) < bytes) lo = mid + 1; else hi = mid;
    }
    if (binning_bytes_for(lo * kCapQuantum) == bytes) {
        *C = lo * kCapQuantum;
        return true;
    }
    *C = (size_t)R;
    return binning_bytes_for((size_t)R) == bytes;
}

// Backward scratch: R per-instance records, P per-Gaussian sums, the live list (the records' content
// bytes are in the binning buffer).
void carve_recs(char* base, size_t R, size_t P, gsr::GradRecs* recs, gsr::GradRecs* sums, uint32_t** live,
                uint32_t** live_count, size_t* total) {
    using namespace gsr;
    Carver c{base, 0};
    {  // interleaved 48-byte records (gsr_common.h kRecAB / kRecC)
        float4* r48 = c.take<float4>(3 * R);
        recs->a = r48;
        recs->b = r48 + 1;
        recs->c = reinterpret_cast<float2*>(r48 + 2);
    }
    recs->flag = nullptr;  // in the binning buffer (BinningState::rec_flag)
    // (per Gaussian, gauss_reduce's; the atomic backward reads its accumulator rows instead)
    sums->a = c.take<float4>(P);
    sums->b = c.take<float4>(P);
    sums->c = c.take<float2>(P);
    sums->flag = nullptr;
    // the Gaussians with a gradient (gauss_reduce appends, gauss_bwd walks), kLiveShards shards
    *live = c.take<uint32_t>((size_t)kLiveShards * live_list_cap((uint32_t)P));
    *live_count = c.take<uint32_t>((size_t)kLiveShards * kLiveCntStride);
    *total = align_up(c.off);
}

// ---- runtime options (include/gsr.h gsr_option_set) ------------------------------
// The library's alternative kernel paths.  Each default comes from GSR_<NAME> in the environment
// at first use; gsr_option_set changes it for later calls (tests/test_gpu_options.py runs every
// path against the oracle).
constexpr uint32_t kFusedFillBlocks = 256;  // one-wave fill blocks in render_bwd's launch (the side-stream kernel: 64 x 4 waves)
// "near_mass": near-first binning (binning.hip) -- only the Gaussians in front of the depth at which the
// screen-averaged opacity mass reaches this value get keys and are sorted; 0 = off.  Capacity-hinted
// forwards with the fused scan only.
// "bwd_atomic": the render backward adds each instance's sums into per-Gaussian rows with float atomics
// (render.hip ATOMIC) and gauss_bwd lists the touched Gaussians itself, instead of per-instance records summed
// by gauss_reduce (deterministic).  The forward zeroes the rows when the option is on at forward time and
// marks its buffer (geom_mark below); a backward adds atomically iff the option is on and its buffer is marked.
constexpr uint32_t kFwdFillBlocks = 256;  // one-wave blocks zeroing the accumulators in render_fwd's launch (a multiple of 8)
static_assert(kFwdFillBlocks % 8 == 0, "the forward's fill blocks keep the tiles' XCD mapping");
enum Opt {
    OPT_FUSED_BIN = 0, OPT_FWD_QUADS, OPT_BWD_SEG_CK, OPT_HOST_TOTAL, OPT_ZERO_FILL, OPT_LIVE_LIST, OPT_SORT_PREFIX,
    OPT_COUNT_WAIT, OPT_BWD_GRID, OPT_BWD_ATOMIC, OPT_NEAR_MASS, OPT_TOUCHED_RUN, OPT_COUNT
};
struct OptionSpec {
    const char* name;
    const char* env;
    int def, lo, hi;
};
const OptionSpec kOptions[OPT_COUNT] = {
    {"fused_bin", "GSR_FUSED_BIN", 1, 0, 1},
    {"fwd_quads", "GSR_FWD_QUADS", 2, 2, 4},
    {"bwd_seg_ck", "GSR_BWD_SEG_CK", 1, 1, 1 << 20},
    {"host_total", "GSR_HOST_TOTAL", 1, 0, 1},
    {"zero_fill", "GSR_ZERO_FILL", 3, 0, 3},
    {"live_list", "GSR_LIVE_LIST", 1, 0, 1},
    {"sort_prefix", "GSR_SORT_PREFIX", 1024, 0, (int)gsr::kSortPrefixMax},
    {"count_wait", "GSR_COUNT_WAIT", 2, 0, 2},
    {"bwd_grid", "GSR_BWD_GRID", 0, 0, 2},
    {"bwd_atomic", "GSR_BWD_ATOMIC", 1, 0, 1},
    {"near_mass", "GSR_NEAR_MASS", 30, 0, 1 << 20},
    {"touched_run", "GSR_TOUCHED_RUN", 0, 0, 32},
};
std::atomic<int> g_opt[OPT_COUNT];
std::once_flag g_opt_once;

void options_init() {
    std::call_once(g_opt_once, [] {
        for (int i = 0; i < OPT_COUNT; i++) {
            const OptionSpec& o = kOptions[i];
            int v = o.def;
            if (const char* e = getenv(o.env)) {
                const int x = atoi(e);
                // out-of-range values clamp (a huge GSR_BWD_SEG_CK means "one unit per tile")
                v = x < o.lo ? o.lo : x > o.hi ? o.hi : x;
                if (i == OPT_FWD_QUADS) v = x == 4 ? 4 : 2;
            }
            g_opt[i].store(v, std::memory_order_relaxed);
        }
    });
}

// Per-thread overrides (gsr_option_set_thread): kOptNone where the process-wide value applies.
constexpr int kOptNone = INT_MIN;
thread_local int t_opt[OPT_COUNT] = {kOptNone, kOptNone, kOptNone, kOptNone, kOptNone, kOptNone, kOptNone, kOptNone,
                                     kOptNone, kOptNone, kOptNone, kOptNone};
static_assert(OPT_COUNT == 12, "one kOptNone per option above");

int option(int id) {
    if (t_opt[id] != kOptNone) return t_opt[id];
    options_init();
    return g_opt[id].load(std::memory_order_relaxed);
}

int option_index(const char* name) {
    if (!name) return -1;
    for (int i = 0; i < OPT_COUNT; i++)
        if (strcmp(name, kOptions[i].name) == 0) return i;
    return -1;
}

// What each geometry buffer's last forward left for its backwards: whether it zeroed the atomic backward's
// accumulator rows ("bwd_atomic" on at forward time) and whether its K3 wrote the record path's inputs (record
// starts, zeroed content bits; skipped when the forward zeroed the rows).  A
// backward adds atomically only into a zeroed buffer, and before a record-path backward of a buffer without
// record inputs it writes them (launch_rec_prep).  A buffer the library never saw (copied in) is neither: the
// record path, after the prep.  Every forward re-marks its buffer, so an address the caching allocator hands
// out again carries its latest forward's state.  Bounded: past kGeomMarksMax entries the table starts over
// (a miss costs a prep, never a wrong result).
struct GeomMark {
    const void* buf;
    bool zeroed, recs;
    bool long_lists;  // the frame's mean tile list is long (kLongMeanList): few of its Gaussians are touched
};
std::mutex g_mark_mu;
std::vector<GeomMark> g_marks;
constexpr size_t kGeomMarksMax = 4096;

void geom_mark(const void* geom_buffer, bool zeroed, bool recs, bool long_lists) {
    std::lock_guard<std::mutex> lk(g_mark_mu);
    for (auto& m : g_marks)
        if (m.buf == geom_buffer) {
            m.zeroed = zeroed;
            m.recs = recs;
            m.long_lists = long_lists;
            return;
        }
    if (!zeroed && !recs) return;  // (absent = neither)
    if (g_marks.size() >= kGeomMarksMax) g_marks.clear();
    g_marks.push_back(GeomMark{geom_buffer, zeroed, recs, long_lists});
}

void geom_forget(const void* geom_buffer) {
    std::lock_guard<std::mutex> lk(g_mark_mu);
    for (size_t i = 0; i < g_marks.size(); i++)
        if (g_marks[i].buf == geom_buffer) {
            g_marks[i] = g_marks.back();
            g_marks.pop_back();
            return;
        }
}

GeomMark geom_marked(const void* geom_buffer) {
    std::lock_guard<std::mutex> lk(g_mark_mu);
    for (const auto& m : g_marks)
        if (m.buf == geom_buffer) return m;
    return GeomMark{geom_buffer, false, false, false};
}

// A frame whose mean tile list holds at least this many entries is a "long-list" frame: near-first binning
// applies (below) and the atomic backward lists its touched Gaussians over longer runs (few are touched).
constexpr size_t kLongMeanList = 2048;

// K2 folded into K3 in capacity mode.
bool fused_binning_mode() { return option(OPT_FUSED_BIN) != 0; }

// The reachable-prefix sort of long lists ("sort_prefix" option, binning.hip K4) for a binning
// buffer of capacity C: on when the frame's lists are long -- mean length >= 2 L -- where sorting
// only their first L entries saves most of K4 (5M@4K: tile_sort 0.70 -> 0.49 ms); off for shorter
// lists, where it saves nothing and the two redo launches cost ~8 us (1M@1080p, r3c).  Census runs
// sort whole lists (a redone tile's first pass would be counted twice).  The results are the same
// either way.
// L <= kSortPrefixMax (the option's range): the prefix kernel's LDS holds 2 kSortPrefixMax keys, so a
// prefix plus the rest of its last bucket fits (a longer one would send every long list to the
// global-memory fallback sort).
uint32_t sort_prefix_for(size_t C, uint32_t tiles, uint32_t L) {
    L = std::min(L, gsr::kSortPrefixMax);
    if (!L || g_census || tiles == 0) return 0u;
    return C / tiles >= 2ull * L ? L : 0u;
}

// Per (host thread, device): a pinned 8-byte slot that num_rendered is copied into and the
// event recorded behind that copy.  The host waits on the event -- i.e. for the binning
// counts -- and not for the whole stream, so the render kernels queued behind the copy keep
// the GPU busy while the host returns to Python and queues the backward.
// The slot is coherent and mapped, and by default K2 stores the count into it itself
// (`dev`), so no copy is queued behind K2; the "host_total" option 0 selects the copy.
struct TotalReadback {
    unsigned long long* host = nullptr;
    unsigned long long* mapped = nullptr;  // device view of `host`
    unsigned long long* dev = nullptr;     // `mapped` when the kernels store the count, null: copy instead
    hipEvent_t ev = nullptr;
};
bool host_total_store() { return option(OPT_HOST_TOTAL) != 0; }
int total_readback(TotalReadback** out, bool kernel_store) {
    constexpr int kMaxDevices = 64;
    thread_local TotalReadback slots[kMaxDevices];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices)
        return fail(GSR_ERR_HIP, "num_rendered readback: no current device");
    TotalReadback& r = slots[dev];
    if (!r.host) {
        // always mapped + coherent, so the "host_total" option can switch between the kernels'
        // own store (dev) and a queued copy (readback_dev() == null) from one call to the next
        void* h = nullptr;
        if (hipHostMalloc(&h, sizeof(unsigned long long), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
            return fail(GSR_ERR_HIP, "num_rendered readback: hipHostMalloc failed");
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
            (void)hipHostFree(h);
            return fail(GSR_ERR_HIP, "num_rendered readback: hipHostGetDevicePointer failed");
        }
        if (hipEventCreateWithFlags(&r.ev, hipEventDisableTiming) != hipSuccess) {
            (void)hipHostFree(h);
            return fail(GSR_ERR_HIP, "num_rendered readback: hipEventCreate failed");
        }
        r.host = (unsigned long long*)h;
        r.mapped = (unsigned long long*)d;
    }
    r.dev = kernel_store ? r.mapped : nullptr;
    *out = &r;
    return GSR_OK;
}

// The forward's wait for its instance count ("count_wait" option).  1: poll the event from this
// thread (up to kCountSpinMs, then block) -- the count lands ~0.6 ms after the call starts, while
// the GPU still has the previous backward and this forward's binning to run, and a blocking wait
// sleeps until the completion interrupt wakes the thread; on a busy host that wake-up was seen to
// take 2 ms (bench slow_steps, r3y4), idling a GPU whose queue holds only the 0.27 ms of sort and
// render behind the count.  0: hipEventSynchronize (HIP's short active wait, then the interrupt).
// The poll spins for kCountSpinUs, then yields the core between queries (std::this_thread::yield:
// returns at once when nothing else wants the core, so a lone rank still sees the count within a
// query's latency, while eight ranks per node plus RCCL proxy and loader threads get the cores
// they need), and after kCountSpinMs falls back to the blocking wait.
constexpr int kCountSpinMs = 20;
constexpr int kCountSpinUs = 100;
hipError_t wait_count_event(hipEvent_t ev, bool poll) {
    if (poll) {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            const hipError_t q = hipEventQuery(ev);
            if (q != hipErrorNotReady) return q;
            const auto dt = std::chrono::steady_clock::now() - t0;
            if (dt > std::chrono::milliseconds(kCountSpinMs)) break;
            if (dt > std::chrono::microseconds(kCountSpinUs)) std::this_thread::yield();
        }
    }
    return hipEventSynchronize(ev);
}

// "count_wait" 2: poll the mapped count slot until it leaves `pending` (the kernel's system-scope
// store), with the same spin-then-yield pacing; after kCountSlotMs the stream itself is waited for
// (a stalled or faulted stream then reports its error instead of the poll spinning on).
constexpr int kCountSlotMs = 2000;
hipError_t wait_count_slot(const unsigned long long* slot, unsigned long long pending, hipStream_t stream) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        if (__atomic_load_n(slot, __ATOMIC_ACQUIRE) != pending) return hipSuccess;
        const auto dt = std::chrono::steady_clock::now() - t0;
        if (dt > std::chrono::milliseconds(kCountSlotMs)) break;
        if (dt > std::chrono::microseconds(kCountSpinUs)) std::this_thread::yield();
    }
    return hipStreamSynchronize(stream);
}

// Forwards whose capacity hint was too small (the binning stage was redone), for gsr_forward_rebuilds().
std::atomic<long long> g_rebuilds{0};
// Host-side statistics (gsr_host_stats): time the forwards waited for their instance count, and
// the host time of whole forward / backward calls.
struct HostStat {
    std::atomic<long long> ns{0}, calls{0}, max_ns{0};
    void add(long long v) {
        ns.fetch_add(v, std::memory_order_relaxed);
        calls.fetch_add(1, std::memory_order_relaxed);
        long long prev = max_ns.load(std::memory_order_relaxed);
        while (v > prev && !max_ns.compare_exchange_weak(prev, v, std::memory_order_relaxed)) {}
    }
    void reset() {
        ns.store(0, std::memory_order_relaxed);
        calls.store(0, std::memory_order_relaxed);
        max_ns.store(0, std::memory_order_relaxed);
    }
};
HostStat g_wait, g_fwd_host, g_bwd_host;
struct HostTimer {  // adds the scope's host time to a HostStat
    HostStat& st;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    explicit HostTimer(HostStat& s) : st(s) {}
    ~HostTimer() {
        st.add((long long)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0)
                   .count());
    }
};

void* call_alloc(gsr_alloc_fn fn, void* ctx, size_t bytes) {
    if (!fn) return nullptr;
    return fn(ctx, bytes ? bytes : 1);
}

}  // namespace

extern "C" {

const char* gsr_last_error(void) { return g_err; }

const char* gsr_version(void) { return "gsr 0.2.0 gfx950"; }

#ifndef GSR_BUILD_ID
#define GSR_BUILD_ID "unknown"
#endif
const char* gsr_build_id(void) { return GSR_BUILD_ID; }

long long gsr_forward_rebuilds(void) { return g_rebuilds.load(std::memory_order_relaxed); }

int gsr_host_stats(double* values, int n, int reset) {
    const HostStat* st[3] = {&g_wait, &g_fwd_host, &g_bwd_host};
    for (int k = 0; k < 3; k++)
        for (int j = 0; j < 3; j++) {
            const int i = 3 * k + j;
            if (!values || i >= n) continue;
            values[i] = j == 0 ? (double)st[k]->calls.load(std::memory_order_relaxed)
                               : (double)(j == 1 ? st[k]->ns : st[k]->max_ns).load(std::memory_order_relaxed) * 1e-6;
        }
    if (reset)
        for (auto* p : {&g_wait, &g_fwd_host, &g_bwd_host}) p->reset();
    return GSR_OK;
}

int gsr_option_set(const char* name, int value) {
    g_err[0] = 0;
    const int i = option_index(name);
    if (i < 0) return fail(GSR_ERR_ARGUMENT, "option_set: unknown option '%s'", name ? name : "(null)");
    const OptionSpec& o = kOptions[i];
    if (value < o.lo || value > o.hi || (i == OPT_FWD_QUADS && value != 2 && value != 4))
        return fail(GSR_ERR_ARGUMENT, "option_set: %s = %d out of range [%d, %d]", name, value, o.lo, o.hi);
    options_init();
    g_opt[i].store(value, std::memory_order_relaxed);
    return GSR_OK;
}

int gsr_option_get(const char* name) {
    const int i = option_index(name);
    return i < 0 ? -1 : option(i);
}

int gsr_option_set_thread(const char* name, int value) {
    g_err[0] = 0;
    const int i = option_index(name);
    if (i < 0) return fail(GSR_ERR_ARGUMENT, "option_set_thread: unknown option '%s'", name ? name : "(null)");
    const OptionSpec& o = kOptions[i];
    if (value < o.lo || value > o.hi || (i == OPT_FWD_QUADS && value != 2 && value != 4))
        return fail(GSR_ERR_ARGUMENT, "option_set_thread: %s = %d out of range [%d, %d]", name, value, o.lo, o.hi);
    t_opt[i] = value;
    return GSR_OK;
}

int gsr_option_clear_thread(const char* name) {
    g_err[0] = 0;
    if (!name) {
        for (int i = 0; i < OPT_COUNT; i++) t_opt[i] = kOptNone;
        return GSR_OK;
    }
    const int i = option_index(name);
    if (i < 0) return fail(GSR_ERR_ARGUMENT, "option_clear_thread: unknown option '%s'", name);
    t_opt[i] = kOptNone;
    return GSR_OK;
}

int gsr_geom_forget(const void* geom_buffer) {
    g_err[0] = 0;
    geom_forget(geom_buffer);
    return GSR_OK;
}

int gsr_fused_ssim_forward(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2,
                           float* ssim_map, float* dm_dmu1, float* dm_dsigma1_sq, float* dm_dsigma12, void* stream) {
    g_err[0] = 0;
    if (B < 0 || CH < 0 || H < 0 || W < 0) return fail(GSR_ERR_ARGUMENT, "fused_ssim: negative size");
    const long long planes = (long long)B * CH;
    if (planes == 0 || H == 0 || W == 0) return GSR_OK;
    if (planes > 65535) return fail(GSR_ERR_ARGUMENT, "fused_ssim: B*CH=%lld exceeds 65535 planes", planes);
    if (!img1 || !img2 || !ssim_map) return fail(GSR_ERR_ARGUMENT, "fused_ssim: null pointer");
    const int ndm = (dm_dmu1 != nullptr) + (dm_dsigma1_sq != nullptr) + (dm_dsigma12 != nullptr);
    if (ndm != 0 && ndm != 3) return fail(GSR_ERR_ARGUMENT, "fused_ssim: pass all three derivative maps or none");
    HIP_TRY(gsr::launch_ssim_fwd((int)planes, H, W, C1, C2, img1, img2, ssim_map, dm_dmu1, dm_dsigma1_sq, dm_dsigma12,
                                 (hipStream_t)stream),
            "fused_ssim forward");
    return GSR_OK;
}

int gsr_fused_ssim_backward(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2,
                            const float* dL_dmap, const float* dm_dmu1, const float* dm_dsigma1_sq,
                            const float* dm_dsigma12, float* dL_dimg1, void* stream) {
    (void)C1;  // the derivative maps already carry C1 and C2 (ssim.cu:315-366 does not use them either)
    (void)C2;
    g_err[0] = 0;
    if (B < 0 || CH < 0 || H < 0 || W < 0) return fail(GSR_ERR_ARGUMENT, "fused_ssim: negative size");
    const long long planes = (long long)B * CH;
    if (planes == 0 || H == 0 || W == 0) return GSR_OK;
    if (planes > 65535) return fail(GSR_ERR_ARGUMENT, "fused_ssim: B*CH=%lld exceeds 65535 planes", planes);
    if (!img1 || !img2 || !dL_dmap || !dm_dmu1 || !dm_dsigma1_sq || !dm_dsigma12 || !dL_dimg1)
        return fail(GSR_ERR_ARGUMENT, "fused_ssim backward: null pointer");
    HIP_TRY(gsr::launch_ssim_bwd((int)planes, H, W, img1, img2, dL_dmap, dm_dmu1, dm_dsigma1_sq, dm_dsigma12, dL_dimg1,
                                 (hipStream_t)stream),
            "fused_ssim backward");
    return GSR_OK;
}

int gsr_knn_mean_dist2(int P, const float* points, float* mean_dists, gsr_alloc_fn scratch_alloc, void* scratch_ctx,
                       void* stream_) {
    g_err[0] = 0;
    hipStream_t stream = (hipStream_t)stream_;
    if (P < 0) return fail(GSR_ERR_ARGUMENT, "knn: P must be >= 0");
    if (P == 0) return GSR_OK;
    if (!points || !mean_dists) return fail(GSR_ERR_ARGUMENT, "knn: null pointer");
    const size_t bytes = gsr::knn_scratch_bytes(P);
    void* scratch = call_alloc(scratch_alloc, scratch_ctx, bytes);
    if (!scratch) return fail(GSR_ERR_ALLOC, "knn: scratch allocation of %zu bytes failed", bytes);
    HIP_TRY(gsr::launch_knn(P, points, mean_dists, scratch, stream), "knn");
    // the caller frees the scratch after the call: finish the work first
    HIP_TRY(hipStreamSynchronize(stream), "knn sync");
    return GSR_OK;
}

// ---- SparseGaussianAdam's step (include/gsr_adam.h) -------------------------------
static_assert(GSR_ADAM_MAX_GROUPS == gsr::kAdamMaxGroups, "group table size");

static int adam_launch(const gsr_adam_group* groups, int n_groups, const unsigned char* visible, int N, float b1,
                       float b2, void* stream) {
    using namespace gsr;
    g_err[0] = 0;
    if (n_groups < 0 || n_groups > GSR_ADAM_MAX_GROUPS)
        return fail(GSR_ERR_ARGUMENT, "adam_update: %d parameter groups (0..%d)", n_groups, GSR_ADAM_MAX_GROUPS);
    if (N < 0) return fail(GSR_ERR_ARGUMENT, "adam_update: N must be >= 0");
    if (N == 0 || n_groups == 0) return GSR_OK;
    if (!visible || !groups) return fail(GSR_ERR_ARGUMENT, "adam_update: null pointer");
    AdamArgs a{};
    a.vis = visible;
    a.b1 = b1;
    a.b2 = b2;
    uint32_t blocks = 0;
    auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    for (int k = 0; k < n_groups; k++) {
        const gsr_adam_group& s = groups[k];
        if (s.M <= 0 || s.numel != (long long)N * s.M)
            return fail(GSR_ERR_ARGUMENT, "adam_update: group %d has %lld values, expected N*M = %d*%d", k, s.numel, N,
                        s.M);
        if (s.numel > 0x7fffffffLL)
            return fail(GSR_ERR_ARGUMENT, "adam_update: group %d has more than 2^31-1 values", k);
        if (!s.param || !s.grad || !s.exp_avg || !s.exp_avg_sq)
            return fail(GSR_ERR_ARGUMENT, "adam_update: group %d has a null parameter/state pointer", k);
        AdamGroupDev& G = a.grp[a.n_groups++];
        G.p = s.param; G.g = s.grad; G.m = s.exp_avg; G.v = s.exp_avg_sq;
        G.n = (uint32_t)s.numel;
        G.M = (uint32_t)s.M;
        uint32_t l = 0;
        while ((1u << l) < G.M) l++;
        G.shift = 31 + l;
        G.magic = ((1ull << G.shift) + G.M - 1) / G.M;  // ceil(2^(31+l) / M): exact i / M for i < 2^31
        G.lr = s.lr;
        G.eps = s.eps;
        G.first_block = blocks;
        G.vec = al16(s.param) && al16(s.grad) && al16(s.exp_avg) && al16(s.exp_avg_sq);
        blocks += (G.n + kAdamBlockElems - 1) / kAdamBlockElems;
    }
    HIP_TRY(launch_adam(a, blocks, (hipStream_t)stream), "adam_update");
    return GSR_OK;
}

int gsr_adam_update(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, const unsigned char* visible,
                    float lr, float b1, float b2, float eps, int N, int M, void* stream) {
    const gsr_adam_group g{param, grad, exp_avg, exp_avg_sq, (long long)N * M, M, lr, eps};
    return adam_launch(&g, 1, visible, N, b1, b2, stream);
}

int gsr_adam_update_multi(const gsr_adam_group* groups, int n_groups, const unsigned char* visible, int N, float b1,
                          float b2, void* stream) {
    return adam_launch(groups, n_groups, visible, N, b1, b2, stream);
}

// ---- adaptive density control (include/gsr_densify.h) ------------------------------
int gsr_densify_stats(int P, const float* viewspace_grad, const int* radii, const unsigned char* visible,
                      float* grad_accum, float* denom, float* max_radii2D, void* stream) {
    using namespace gsr;
    g_err[0] = 0;
    if (P < 0) return fail(GSR_ERR_ARGUMENT, "densify_stats: P must be >= 0");
    if (P == 0) return GSR_OK;
    if (viewspace_grad && (!grad_accum || !denom)) return fail(GSR_ERR_ARGUMENT, "densify_stats: null accumulator");
    if (!viewspace_grad && !(radii && max_radii2D))
        return fail(GSR_ERR_ARGUMENT, "densify_stats: nothing to update");
    if (!radii && !visible) return fail(GSR_ERR_ARGUMENT, "densify_stats: need radii or a visibility mask");
    HIP_TRY(launch_densify_stats(P, viewspace_grad, radii, visible, grad_accum, denom, max_radii2D,
                                 (hipStream_t)stream),
            "densify_stats");
    return GSR_OK;
}

unsigned long long gsr_densify_scratch_bytes(int P) { return P > 0 ? gsr::densify_scratch_bytes(P) : 0ull; }

int gsr_densify_plan(int P, const float* grad_accum, const float* denom, const float* opacity, const float* scaling,
                     const gsr_densify_params* prm, void* scratch, unsigned char* split_mask, long long* counts,
                     void* stream) {
    using namespace gsr;
    g_err[0] = 0;
    if (!prm || !counts) return fail(GSR_ERR_ARGUMENT, "densify_plan: null params/counts");
    if (P < 0) return fail(GSR_ERR_ARGUMENT, "densify_plan: P must be >= 0");
    for (int k = 0; k < GSR_DENSIFY_NCOUNTS; k++) counts[k] = 0;
    if (P == 0) return GSR_OK;
    if (!grad_accum || !denom || !opacity || !scaling || !scratch)
        return fail(GSR_ERR_ARGUMENT, "densify_plan: null pointer");
    if (prm->split_n < 1 || prm->split_n > 64) return fail(GSR_ERR_ARGUMENT, "densify_plan: split N = %d", prm->split_n);
    DensifyArgs a{};
    a.P = P;
    a.accum = grad_accum; a.denom = denom; a.opacity = opacity; a.scaling = scaling;
    a.grad_threshold = prm->grad_threshold; a.clone_extent = prm->clone_extent; a.min_opacity = prm->min_opacity;
    a.big_extent = prm->big_extent; a.split_div = prm->split_div; a.use_screen_size = prm->use_screen_size;
    a.split_mask = split_mask;
    densify_carve(scratch, P, a);
    const hipStream_t s = (hipStream_t)stream;
    HIP_TRY(launch_densify_plan(a, s), "densify_plan");
    uint32_t tot[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(tot, a.totals, sizeof(tot), hipMemcpyDeviceToHost, s), "densify_plan counts");
    HIP_TRY(hipStreamSynchronize(s), "densify_plan sync");
    counts[GSR_DENSIFY_KEPT] = tot[0];
    counts[GSR_DENSIFY_CLONES] = tot[1];
    counts[GSR_DENSIFY_CHILDREN] = tot[2];
    counts[GSR_DENSIFY_SPLIT] = tot[3];
    counts[GSR_DENSIFY_TOTAL] = (long long)tot[0] + tot[1] + (long long)prm->split_n * tot[2];
    if (counts[GSR_DENSIFY_TOTAL] > 0x7fffffffLL)
        return fail(GSR_ERR_OVERFLOW, "densify_plan: %lld Gaussians after densification", counts[GSR_DENSIFY_TOTAL]);
    return GSR_OK;
}

int gsr_densify_apply(int P, const void* scratch, const gsr_densify_group* groups, int n_groups,
                      const float* rotation, const float* samples, const int* tmp_radii_in, int* tmp_radii_out,
                      const gsr_densify_params* prm, void* stream) {
    using namespace gsr;
    g_err[0] = 0;
    if (!prm) return fail(GSR_ERR_ARGUMENT, "densify_apply: null params");
    if (P < 0 || n_groups < 0 || n_groups > GSR_DENSIFY_MAX_GROUPS)
        return fail(GSR_ERR_ARGUMENT, "densify_apply: P = %d, %d groups (0..%d)", P, n_groups, GSR_DENSIFY_MAX_GROUPS);
    if (P == 0) return GSR_OK;
    if (!scratch || (n_groups > 0 && !groups)) return fail(GSR_ERR_ARGUMENT, "densify_apply: null pointer");
    if ((tmp_radii_in == nullptr) != (tmp_radii_out == nullptr))
        return fail(GSR_ERR_ARGUMENT, "densify_apply: tmp_radii in and out must both be given or both be null");
    DensifyArgs d{};
    densify_carve(const_cast<void*>(scratch), P, d);
    const hipStream_t s = (hipStream_t)stream;
    uint32_t tot[4] = {0, 0, 0, 0};  // the plan's totals (a tiny synchronous read; the plan already synchronised)
    HIP_TRY(hipMemcpyAsync(tot, d.totals, sizeof(tot), hipMemcpyDeviceToHost, s), "densify_apply counts");
    HIP_TRY(hipStreamSynchronize(s), "densify_apply sync");
    if ((unsigned long long)tot[0] + tot[1] + (unsigned long long)prm->split_n * tot[2] == 0)
        return GSR_OK;  // everything pruned: the new arrays are empty
    if (tot[3] > 0 && tot[2] > 0 && !samples)
        return fail(GSR_ERR_ARGUMENT, "densify_apply: %u split Gaussians but no samples", tot[3]);
    auto launch = [&](const void* src, void* dst, const void* sm, const void* sv, void* dm, void* dv, int width,
                      int role, const char* what) -> int {
        if (width <= 0) return fail(GSR_ERR_ARGUMENT, "densify_apply: %s width %d", what, width);
        if ((size_t)P * (size_t)width > 0x7fffffffull)
            return fail(GSR_ERR_ARGUMENT, "densify_apply: %s has more than 2^31-1 values", what);
        if (!src || !dst) return fail(GSR_ERR_ARGUMENT, "densify_apply: %s null array", what);
        if ((sm == nullptr) != (dm == nullptr) || (sv == nullptr) != (dv == nullptr) || (sm == nullptr) != (sv == nullptr))
            return fail(GSR_ERR_ARGUMENT, "densify_apply: %s Adam state pointers must all be given or all be null",
                        what);
        if (role == GSR_DENSIFY_XYZ && (width != 3 || !rotation))
            return fail(GSR_ERR_ARGUMENT, "densify_apply: the xyz group needs width 3 and the rotations");
        if (role == GSR_DENSIFY_SCALING && width != 3)
            return fail(GSR_ERR_ARGUMENT, "densify_apply: the scaling group needs width 3");
        if (role < GSR_DENSIFY_COPY || role > GSR_DENSIFY_SCALING)
            return fail(GSR_ERR_ARGUMENT, "densify_apply: %s role %d", what, role);
        DensifyApplyArgs a{};
        a.src = (const uint32_t*)src; a.dst = (uint32_t*)dst;
        a.src_m = (const uint32_t*)sm; a.src_v = (const uint32_t*)sv; a.dst_m = (uint32_t*)dm; a.dst_v = (uint32_t*)dv;
        a.n = (uint32_t)((size_t)P * width);
        a.width = (uint32_t)width;
        uint32_t l = 0;
        while ((1u << l) < a.width) l++;
        a.shift = 31 + l;
        a.magic = ((1ull << a.shift) + a.width - 1) / a.width;  // exact t / width for t < 2^31
        a.role = role;
        a.rows = d.rows;
        a.rotation = rotation;
        a.samples = samples;
        a.n_split = tot[3];
        a.n_children = tot[2];
        a.split_n = prm->split_n;
        a.split_div = prm->split_div;
        HIP_TRY(launch_densify_apply(a, s), "densify_apply");
        return GSR_OK;
    };
    for (int k = 0; k < n_groups; k++) {
        const gsr_densify_group& g = groups[k];
        if (int rc = launch(g.src, g.dst, g.src_exp_avg, g.src_exp_avg_sq, g.dst_exp_avg, g.dst_exp_avg_sq, g.width,
                            g.role, "group"))
            return rc;
    }
    if (tmp_radii_in)
        if (int rc = launch(tmp_radii_in, tmp_radii_out, nullptr, nullptr, nullptr, nullptr, 1, GSR_DENSIFY_COPY,
                            "tmp_radii"))
            return rc;
    return GSR_OK;
}

int gsr_census_set(void* device_counters) {
    g_census = reinterpret_cast<unsigned long long*>(device_counters);
    return GSR_OK;
}

int gsr_profile_enable(int stage_mask) {
    std::lock_guard<std::mutex> lk(g_prof.mu);
    g_prof.mask = (unsigned)stage_mask;
    return GSR_OK;
}

void gsr_profile_reset(void) {
    std::lock_guard<std::mutex> lk(g_prof.mu);
    for (auto& p : g_prof.pending) {
        g_prof.pool.push_back(p.a);
        g_prof.pool.push_back(p.b);
    }
    g_prof.pending.clear();
    for (int i = 0; i < ST_COUNT; i++) {
        g_prof.total_ms[i] = 0;
        g_prof.calls[i] = 0;
    }
}

int gsr_profile_collect(double* total_ms, long long* calls, int max_stages) {
    std::lock_guard<std::mutex> lk(g_prof.mu);
    for (auto& p : g_prof.pending) {
        (void)hipEventSynchronize(p.b);
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            g_prof.total_ms[p.stage] += ms;
            g_prof.calls[p.stage] += 1;
        }
        g_prof.pool.push_back(p.a);
        g_prof.pool.push_back(p.b);
    }
    g_prof.pending.clear();
    for (int i = 0; i < ST_COUNT && i < max_stages; i++) {
        if (total_ms) total_ms[i] = g_prof.total_ms[i];
        if (calls) calls[i] = g_prof.calls[i];
    }
    return ST_COUNT;
}

const char* gsr_profile_stage_name(int stage) {
    return (stage >= 0 && stage < ST_COUNT) ? kStageNames[stage] : "";
}

int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     unsigned char* present, void* stream) {
    (void)projmatrix;  // checkFrustum computes the projection but only tests view-space z
    g_err[0] = 0;
    if (P < 0) return fail(GSR_ERR_ARGUMENT, "mark_visible: P must be >= 0");
    if (P == 0) return GSR_OK;
    if (!means3D || !viewmatrix || !present) return fail(GSR_ERR_ARGUMENT, "mark_visible: null pointer");
    HIP_TRY(gsr::launch_mark_visible(P, means3D, viewmatrix, reinterpret_cast<bool*>(present), (hipStream_t)stream),
            "mark_visible");
    return GSR_OK;
}

namespace {
int forward_impl(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                 gsr_alloc_fn image_alloc, void* image_ctx, int P, int D, int M, const float* background, int width,
                 int height, const float* means3D, const float* dc, const float* shs, const float* colors_precomp,
                 const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                 const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix, const float* cam_pos,
                 float tan_fovx, float tan_fovy, int prefiltered, float* out_color, float* out_invdepth,
                 int antialiasing, int* radii, int debug, void* stream_, int* num_rendered, int capacity_hint,
                 int* binning_capacity, bool quantized = true) {
    using namespace gsr;
    HostTimer host_time(g_fwd_host);
    g_err[0] = 0;
    hipStream_t stream = (hipStream_t)stream_;
    // every option is read ONCE per call: gsr_option_set may run on another thread, and the launches
    // of one forward (K4's prefix and the redo, the render's part protocol, the work list's segment
    // length) must agree with each other
    const int opt_quads = option(OPT_FWD_QUADS), opt_seg_ck = option(OPT_BWD_SEG_CK);
    const uint32_t opt_prefix = (uint32_t)option(OPT_SORT_PREFIX);
    const bool opt_fused = fused_binning_mode(), opt_host_total = host_total_store();
    const int opt_count_wait = option(OPT_COUNT_WAIT);
    const bool opt_atomic = option(OPT_BWD_ATOMIC) != 0;
    // K3 writes the record path's inputs only when this forward's backwards may take it without a prep
    const bool k3_recs = !opt_atomic;
    const int opt_near_mass = option(OPT_NEAR_MASS);
    // _ex / _dc forwards lay the binning buffer out for a multiple of kCapQuantum (the backward
    // recovers it from the buffer's size); gsr_rasterize_forward keeps the exact C = R layout
    const auto capacity_for = [quantized](size_t c) {
        const size_t q = quantize_capacity(c);
        return quantized && q <= (size_t)INT_MAX ? q : c;
    };
    if (num_rendered) *num_rendered = 0;
    if (binning_capacity) *binning_capacity = 0;
    if (P < 0 || width <= 0 || height <= 0)
        return fail(GSR_ERR_ARGUMENT, "rasterize_forward: invalid sizes P=%d W=%d H=%d", P, width, height);
    if (P >= kMaxGaussians)
        return fail(GSR_ERR_ARGUMENT, "rasterize_forward: P=%d exceeds the tile-list entry limit %d", P,
                    kMaxGaussians - 1);
    if (P == 0) return GSR_OK;  // RI/rasterize_points.cu:108: nothing is launched
    if (!means3D || !opacities || !viewmatrix || !projmatrix || !background || !out_color || !out_invdepth || !radii)
        return fail(GSR_ERR_ARGUMENT, "rasterize_forward: missing required input");
    if (!colors_precomp && !shs && !dc)
        return fail(GSR_ERR_ARGUMENT, "rasterize_forward: provide either SHs or precomputed colours");
    if (dc && M > 0 && !shs) return fail(GSR_ERR_ARGUMENT, "rasterize_forward: %d rest SH coefficients but no shs", M);
    if (dc) M += 1;  // split layout: M counted the rest; the kernels see dc as coefficient 0
    if (!cov3D_precomp && (!scales || !rotations))
        return fail(GSR_ERR_ARGUMENT, "rasterize_forward: provide scales+rotations or a precomputed covariance");
    if (!colors_precomp && (D < 0 || D > 3 || (D + 1) * (D + 1) > M))
        return fail(GSR_ERR_ARGUMENT, "rasterize_forward: SH degree %d needs %d coefficients, got %d", D,
                    (D + 1) * (D + 1), M);
    if (!colors_precomp && !cam_pos) return fail(GSR_ERR_ARGUMENT, "rasterize_forward: campos required for SHs");

    const float focal_y = height / (2.0f * tan_fovy);  // CR/rasterizer_impl.cu:253-254
    const float focal_x = width / (2.0f * tan_fovx);
    const uint32_t gx = (width + kTile - 1) / kTile, gy = (height + kTile - 1) / kTile;
    const uint32_t tiles = gx * gy;
    if (gx > 65535u || gy > 65535u)
        return fail(GSR_ERR_ARGUMENT, "rasterize_forward: image of %dx%d has more than 65535 tile columns/rows",
                    width, height);
    // the binning's instance walk divides tile offsets inside a rectangle in fp32 (exact below 2^21,
    // binning.hip for_each_instance): a 536-Mpx frame, far beyond any camera
    constexpr size_t kMaxTiles = size_t(1) << 21;
    if ((size_t)gx * gy >= kMaxTiles)
        return fail(GSR_ERR_ARGUMENT, "rasterize_forward: image of %dx%d has %zu tiles (the limit is %zu)", width,
                    height, (size_t)gx * gy, kMaxTiles - 1);

    size_t geom_bytes = 0, img_bytes = 0;
    carve_geom(nullptr, P, gx, gy, &geom_bytes);
    char* gbase = (char*)call_alloc(geom_alloc, geom_ctx, geom_bytes);
    if (!gbase) return fail(GSR_ERR_ALLOC, "rasterize_forward: geometry buffer allocation failed");
    GeomState geom = carve_geom(gbase, P, gx, gy, &geom_bytes);
    geom_mark(gbase, false, false, false);  // (set below once the binning and the render's fill blocks are queued)
    carve_image(nullptr, width, height, tiles, &img_bytes);
    char* ibase = (char*)call_alloc(image_alloc, image_ctx, img_bytes);
    if (!ibase) return fail(GSR_ERR_ALLOC, "rasterize_forward: image buffer allocation failed");
    ImageState img = carve_image(ibase, width, height, tiles, &img_bytes);

    if (prefiltered) HIP_TRY(hipMemsetAsync(geom.status, 0, 4 * sizeof(uint32_t), stream), "status init");
    {
        StageScope sc(ST_PREPROCESS, stream);
        PreprocessArgs pa{};
        pa.P = P; pa.D = D; pa.M = M; pa.W = width; pa.H = height;
        pa.means3D = means3D; pa.scales = scales; pa.scale_modifier = scale_modifier; pa.rotations = rotations;
        pa.opacities = opacities; pa.shs = colors_precomp || M <= (dc ? 1 : 0) ? nullptr : shs;
        pa.dc = colors_precomp ? nullptr : dc; pa.cov3D_precomp = cov3D_precomp;
        pa.colors_precomp = colors_precomp; pa.viewmatrix = viewmatrix; pa.projmatrix = projmatrix;
        pa.campos = cam_pos; pa.tan_fovx = tan_fovx; pa.tan_fovy = tan_fovy; pa.focal_x = focal_x;
        pa.focal_y = focal_y; pa.gx = gx; pa.gy = gy; pa.prefiltered = prefiltered; pa.antialiasing = antialiasing;
        pa.footprint_cull = (width < 32000 && height < 32000) ? 1 : 0;
        pa.radii = radii; pa.geom = geom;
        pa.zero = geom.tile_cnt;  // tile, cell and near counters and the depth-mass histogram (binning.hip), contiguous
        pa.zero_n = (uint32_t)bin_zero_words(tiles, bin_cell_count(gx, gy));
        HIP_TRY(launch_preprocess(pa, stream), "preprocess");
    }
    if (int rc = check_debug(debug, stream, "preprocess")) return rc;
    if (prefiltered) {
        uint32_t st = 0;
        HIP_TRY(hipMemcpyAsync(&st, geom.status, sizeof(uint32_t), hipMemcpyDeviceToHost, stream), "status copy");
        HIP_TRY(hipStreamSynchronize(stream), "status sync");
        if (st & 1u)
            return fail(GSR_ERR_PREFILTERED,
                        "Point is filtered although prefiltered is set. This shouldn't happen! (CR/auxiliary.h:184)");
    }
    // exact mode: counts first (ranges unclamped), then the host reads R
    const size_t kNoCap = ~(size_t)0;
    TotalReadback* rb = nullptr;
    if (int rc = total_readback(&rb, opt_host_total)) return rc;
    // capacity mode: the binning buffer's capacity, known up front (the ranges are clamped to it)
    const size_t C_hint = capacity_hint > 0 ? capacity_for((size_t)capacity_hint) : 0;
    // capacity mode with LDS cursors: K2 folded into K3 (binning.hip FusedScan)
    const bool fused = capacity_hint > 0 && bin_fused_ok(tiles) && opt_fused;
    // near-first binning (binning.hip): the depth cut's target, mass x kMassScale over the image.  Only for frames
    // whose lists are long (a mean of kNearMinMeanList entries by the capacity hint, the reachable-prefix sort's
    // regime): there the blend reaches a small part of each list and the cut pays; with short lists (1M@1080p:
    // 973) the frame's mass stays under the target anyway, and the redo chain's launches (far fill, whole
    // sort, redo render: ~6 us when empty) would only cost (r5d: 0.7305 -> 0.7372-0.7404 ms with no cut made)
    constexpr size_t kNearMinMeanList = kLongMeanList;
    const unsigned long long near_target =
        fused && opt_near_mass > 0 && bin_near_ok(tiles) && C_hint >= kNearMinMeanList * (size_t)tiles
            ? (unsigned long long)opt_near_mass * (unsigned long long)kMassScale * (unsigned long long)width * height
            : 0ull;
    const bool near_first = near_target > 0;
    // "count_wait" 2 (capacity mode, the kernels storing the count into the mapped slot): no event
    // behind the count -- the host polls the slot itself, reset to a sentinel before the launch that
    // stores it, so the stream carries no marker (an event's marker left the GPU idle ~6 us between
    // the scatter and the sort, r4a trace)
    const bool poll_slot = opt_count_wait == 2 && capacity_hint > 0 && rb->dev;
    constexpr unsigned long long kSlotPending = ~0ull;
    if (poll_slot) __atomic_store_n(rb->host, kSlotPending, __ATOMIC_RELEASE);
    {
        StageScope sc(ST_BIN_COUNT, stream);
        HIP_TRY(launch_bin_count(P, geom, gx, gy, img.ranges, capacity_hint > 0 ? C_hint : kNoCap,
                                 fused ? nullptr : rb->dev, stream, fused, near_target),
                "bin_count");
    }
    if (int rc = check_debug(debug, stream, "bin_count")) return rc;

    // Scatter + tile sort + render into a binning buffer of capacity C.  In exact mode
    // C = R is read back first -- the reference's one host synchronisation
    // (CR/rasterizer_impl.cu:313).  In capacity mode (capacity_hint > 0) nothing waits
    // for the host: every stage is queued, then the host waits for the copy of R queued
    // right behind K2 (not for the render behind it), and if R exceeds C the lists are
    // rebuilt into a buffer of exactly R.
    // mark num_rendered (K2 stores it into the host slot, or a copy is queued); wait_total()
    // waits for that mark only
    auto queue_total = [&]() -> int {
        if (poll_slot) return GSR_OK;
        if (!rb->dev)
            HIP_TRY(hipMemcpyAsync(rb->host, geom.total, sizeof(*rb->host), hipMemcpyDeviceToHost, stream),
                    "num_rendered copy");
        HIP_TRY(hipEventRecord(rb->ev, stream), "num_rendered event");
        return GSR_OK;
    };
    auto wait_total = [&](unsigned long long* total) -> int {
        hipError_t we;
        {
            HostTimer ht(g_wait);
            we = poll_slot ? wait_count_slot(rb->host, kSlotPending, stream)
                           : wait_count_event(rb->ev, opt_count_wait != 0);
        }
        HIP_TRY(we, "num_rendered sync");
        *total = __atomic_load_n(rb->host, __ATOMIC_ACQUIRE);
        if (*total == kSlotPending)
            return fail(GSR_ERR_HIP, "rasterize_forward: the stream finished without storing the instance count");
        if (*total > (unsigned long long)INT_MAX)
            return fail(GSR_ERR_OVERFLOW, "rasterize_forward: %llu tile instances exceed INT_MAX", *total);
        return GSR_OK;
    };
    auto bin_and_render = [&](size_t C, bool fused_now) -> int {
        size_t bin_bytes = 0;
        carve_binning(nullptr, C, &bin_bytes);
        char* bbase = (char*)call_alloc(binning_alloc, binning_ctx, bin_bytes);
        if (!bbase) return fail(GSR_ERR_ALLOC, "rasterize_forward: binning buffer allocation failed");
        BinningState bin = carve_binning(bbase, C, &bin_bytes);
        const uint32_t prefix = C > 0 ? sort_prefix_for(C, tiles, opt_prefix) : 0u;  // K4 and the redo agree
        {
            // always launched: besides the keys (none when C == 0) it writes every Gaussian's
            // first record index, which the backward's reduction reads even when nothing
            // was rendered (fused: also the ranges, classes and the count)
            StageScope sc(ST_BIN_SCATTER, stream);
            HIP_TRY(launch_bin_scatter(P, geom, gx, gy, bin, C, stream, img.ranges, fused_now ? rb->dev : nullptr,
                                       fused_now, fused_now && near_first, k3_recs),
                    "bin_scatter");
        }
        if (fused_now)
            if (int rc = queue_total()) return rc;
        if (int rc = check_debug(debug, stream, "bin_scatter")) return rc;
        if (C > 0) {
            {
                StageScope sc(ST_TILE_SORT, stream);
                // (near-first binning: K4 sorts each tile's near entries, GeomState::sranges)
                HIP_TRY(launch_tile_sort(tiles, fused_now && near_first ? geom.sranges : img.ranges, geom, bin, C,
                                         stream, fused_now,
                                         (uint32_t)bin_cell_count(gx, gy), prefix),
                        "tile_sort");
            }
            if (int rc = check_debug(debug, stream, "tile_sort")) return rc;
        }
        {
            StageScope sc(ST_RENDER_FWD, stream);
            RenderFwdArgs ra{};
            ra.W = width; ra.H = height; ra.gx = gx; ra.gy = gy; ra.ranges = img.ranges;
            ra.gid_sorted = bin.gid_sorted; ra.rec = geom.rec; ra.bg = background;
            ra.out_color = out_color; ra.out_invdepth = out_invdepth; ra.ckpt = bin.ckpt; ra.img = img;
            ra.unit_cnt = geom.unit_cnt; ra.unit_part = geom.unit_part; ra.unit_full = bin.unit_full;
            ra.full_cap = (uint32_t)unit_full_cap(C);
            ra.tile_join = geom.tile_join;
            ra.seg_ck = opt_seg_ck;
            ra.seg_ck_out = geom.fwd_seg_ck;
            ra.fault = geom.status + 1;
            ra.census = g_census;
            ra.sorted_len = geom.sorted_len;
            ra.redo_flag = geom.redo_flag;
            ra.redo_list = geom.redo_list;
            ra.redo_cnt = geom.redo_cnt;
            // (C == 0: no lists and no K4, so nothing is prefix-sorted and no redo state was reset)
            if (C == 0) ra.sorted_len = nullptr;
            if (opt_atomic) {  // the atomic backward's accumulator rows and touched bits, zeroed beside the render
                ra.acc = geom.acc;
                ra.touched = geom.touched;
                ra.depth_key = geom.depth_key;
                ra.zcut = geom.zcut;
                ra.n_gauss = (uint32_t)P;
                ra.fill_blocks = kFwdFillBlocks;
            }
            HIP_TRY(launch_render_fwd(ra, stream, opt_quads), "render_fwd");
            geom_mark(gbase, opt_atomic, k3_recs, (size_t)C >= kLongMeanList * (size_t)tiles);
            const bool near_now = fused_now && near_first;
            if ((prefix || near_now) && C > 0) {  // the tiles whose walk passed their sorted prefix (usually none)
                if (near_now)  // their far instances first (none emitted by K3); their accumulator rows zeroed
                    HIP_TRY(launch_far_fill(P, geom, gx, tiles, img.ranges, bin, C, true, stream,
                                            opt_atomic ? geom.acc : nullptr),
                            "render_fwd far fill");
                HIP_TRY(launch_tile_sort_redo(tiles, img.ranges, geom, bin, C, stream), "render_fwd redo sort");
                HIP_TRY(launch_render_fwd_redo(ra, stream, opt_quads), "render_fwd redo");
            }
        }
        return check_debug(debug, stream, "render_fwd");
    };

    unsigned long long total = 0;
    size_t C = 0;
    if (!fused)
        if (int rc = queue_total()) return rc;
    if (capacity_hint <= 0) {
        if (int rc = wait_total(&total)) return rc;
        C = capacity_for((size_t)total);
        if (int rc = bin_and_render(C, false)) return rc;
    } else {
        // everything is queued before the host waits, and it waits for the counts only
        C = C_hint;
        if (int rc = bin_and_render(C, fused)) return rc;
        if (int rc = wait_total(&total)) return rc;
        if (total > C) {  // the hint was too small: recount (resets the cursors) and rebuild exactly
            g_rebuilds.fetch_add(1, std::memory_order_relaxed);
            C = capacity_for((size_t)total);
            if (fused)  // (the fused sort re-zeroes the counters only when it ran: C > 0)
                HIP_TRY(hipMemsetAsync(geom.tile_cnt, 0, sizeof(uint32_t) * bin_zero_words(tiles, bin_cell_count(gx, gy)),
                                       stream),
                        "bin counters");
            HIP_TRY(launch_bin_count(P, geom, gx, gy, img.ranges, C, nullptr, stream), "bin_count");
            if (int rc = bin_and_render(C, false)) return rc;
        }
    }
    if (num_rendered) *num_rendered = (int)total;
    if (binning_capacity) *binning_capacity = (int)C;
    return GSR_OK;
}
}  // namespace

int gsr_rasterize_forward(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                          gsr_alloc_fn image_alloc, void* image_ctx, int P, int D, int M, const float* background,
                          int width, int height, const float* means3D, const float* shs, const float* colors_precomp,
                          const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                          const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                          const float* cam_pos, float tan_fovx, float tan_fovy, int prefiltered, float* out_color,
                          float* out_invdepth, int antialiasing, int* radii, int debug, void* stream,
                          int* num_rendered) {
    return forward_impl(geom_alloc, geom_ctx, binning_alloc, binning_ctx, image_alloc, image_ctx, P, D, M, background,
                        width, height, means3D, nullptr, shs, colors_precomp, opacities, scales, scale_modifier, rotations,
                        cov3D_precomp, viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, prefiltered, out_color,
                        out_invdepth, antialiasing, radii, debug, stream, num_rendered, 0, nullptr, false);
}

int gsr_rasterize_forward_ex(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                             gsr_alloc_fn image_alloc, void* image_ctx, int P, int D, int M, const float* background,
                             int width, int height, const float* means3D, const float* shs,
                             const float* colors_precomp, const float* opacities, const float* scales,
                             float scale_modifier, const float* rotations, const float* cov3D_precomp,
                             const float* viewmatrix, const float* projmatrix, const float* cam_pos, float tan_fovx,
                             float tan_fovy, int prefiltered, float* out_color, float* out_invdepth, int antialiasing,
                             int* radii, int debug, void* stream, int* num_rendered, int capacity_hint,
                             int* binning_capacity) {
    return forward_impl(geom_alloc, geom_ctx, binning_alloc, binning_ctx, image_alloc, image_ctx, P, D, M, background,
                        width, height, means3D, nullptr, shs, colors_precomp, opacities, scales, scale_modifier, rotations,
                        cov3D_precomp, viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, prefiltered, out_color,
                        out_invdepth, antialiasing, radii, debug, stream, num_rendered, capacity_hint,
                        binning_capacity);
}

namespace {
// The backward's dense outputs are zero-filled on a side stream that runs beside render_bwd
// (VALU-bound: HBM is two-thirds idle under it); gauss_bwd then writes only the rows of
// Gaussians with a non-zero render gradient (about 14% of a 1M@1080p view).  "zero_fill" option:
// 3 (default) fill blocks in render_bwd's own launch (no events: each fork / join event left the GPU
// idle for 6-7 us, r4a), 1 side stream, 2 main stream right before gauss_bwd, 0 gauss_bwd writes
// every row.
// "live_list": gauss_bwd over the list of Gaussians with a gradient (1, default) or a lane per
// Gaussian (0), when the outputs are zero-filled.
bool live_list_mode() { return option(OPT_LIVE_LIST) != 0; }
int zero_fill_mode() { return option(OPT_ZERO_FILL); }

struct SideStream {
    std::mutex mu;  // one backward at a time per device uses the pair of events
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    bool ok = false;
};

SideStream* side_stream() {
    static SideStream ss[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    SideStream& r = ss[dev];
    std::lock_guard<std::mutex> lk(r.mu);
    if (!r.ok && !r.s) {
        r.ok = hipStreamCreateWithFlags(&r.s, hipStreamNonBlocking) == hipSuccess &&
               hipEventCreateWithFlags(&r.fork, hipEventDisableTiming) == hipSuccess &&
               hipEventCreateWithFlags(&r.join, hipEventDisableTiming) == hipSuccess;
    }
    return r.ok ? &r : nullptr;
}

int backward_impl(int P, int D, int M, int R, const float* background, int width, int height, const float* means3D,
                  const float* dc, const float* shs, const float* colors_precomp, const float* opacities, const float* scales,
                  float scale_modifier, const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                  const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy, const int* radii,
                  void* geom_buffer, void* binning_buffer, void* image_buffer, const float* dL_dpix,
                  const float* dL_dinvdepths, float* dL_dmean2D, float* dL_dconic, float* dL_dopacity,
                  float* dL_dcolor, float* dL_dinvdepth, float* dL_dmean3D, float* dL_dcov3D, float* dL_ddc,
                  float* dL_dsh, float* dL_dscale, float* dL_drot, int antialiasing, int debug, gsr_alloc_fn scratch_alloc,
                  void* scratch_ctx, void* stream_, int binning_capacity, size_t binning_bytes,
                  float* view_block = nullptr) {
    using namespace gsr;
    HostTimer host_time(g_bwd_host);
    g_err[0] = 0;
    hipStream_t stream = (hipStream_t)stream_;
    // view_block: screen-space backward only -- the render-gradient sums, flags and camera go
    // into the block (gsr_rasterize_backward_screen) and the per-Gaussian backward is skipped
    const bool screen = view_block != nullptr;
    if (P < 0 || R < 0 || width <= 0 || height <= 0)
        return fail(GSR_ERR_ARGUMENT, "rasterize_backward: invalid sizes P=%d R=%d W=%d H=%d", P, R, width, height);
    if (P == 0) return GSR_OK;
    if (!geom_buffer || !image_buffer || (R > 0 && !binning_buffer))
        return fail(GSR_ERR_ARGUMENT, "rasterize_backward: missing forward buffers");
    if (!means3D || !opacities || !radii || !dL_dpix || !viewmatrix || !projmatrix || !background || !campos)
        return fail(GSR_ERR_ARGUMENT, "rasterize_backward: missing required pointer");
    if (!screen) {
        if (!dL_dmean2D || !dL_dopacity || !dL_dcolor || !dL_dmean3D || !dL_dcov3D)
            return fail(GSR_ERR_ARGUMENT, "rasterize_backward: missing required output");
        if (!colors_precomp && shs && !dL_dsh)
            return fail(GSR_ERR_ARGUMENT, "rasterize_backward: SH gradient needs dL_dsh");
        if (!colors_precomp && dc && !dL_ddc)
            return fail(GSR_ERR_ARGUMENT, "rasterize_backward: dc gradient needs dL_ddc");
        if (scales && (!rotations || !dL_dscale || !dL_drot))
            return fail(GSR_ERR_ARGUMENT, "rasterize_backward: scale/rotation gradients need outputs");
        if ((dL_dinvdepths == nullptr) != (dL_dinvdepth == nullptr))
            return fail(GSR_ERR_ARGUMENT, "rasterize_backward: dL_dinvdepths and dL_dinvdepth go together");
    }
    if (dc && M > 0 && !shs) return fail(GSR_ERR_ARGUMENT, "rasterize_backward: %d rest SH coefficients but no shs", M);
    if (dc) M += 1;  // as in the forward
    if (!colors_precomp && (shs || dc) && (D < 0 || D > 3 || (D + 1) * (D + 1) > M))
        return fail(GSR_ERR_ARGUMENT, "rasterize_backward: SH degree %d needs %d coefficients, got %d", D,
                    (D + 1) * (D + 1), M);

    const float focal_y = height / (2.0f * tan_fovy);
    const float focal_x = width / (2.0f * tan_fovx);
    const uint32_t gx = (width + kTile - 1) / kTile, gy = (height + kTile - 1) / kTile;
    const uint32_t tiles = gx * gy;
    // the binning buffer is laid out for the capacity the forward used (>= R): given, or
    // recovered from the buffer's size (resolve_capacity)
    size_t C = 0;
    if (!resolve_capacity(R, binning_capacity, binning_bytes, &C))
        return fail(GSR_ERR_ARGUMENT,
                    "rasterize_backward: a binning buffer of %zu bytes matches no layout for R=%d (capacity %d)",
                    binning_bytes, R, binning_capacity);
    if (C < (size_t)R) return fail(GSR_ERR_ARGUMENT, "rasterize_backward: binning capacity %zu < R=%d", C, R);
    size_t tmp = 0;
    GeomState geom = carve_geom((char*)geom_buffer, P, gx, gy, &tmp);
    ImageState img = carve_image((char*)image_buffer, width, height, tiles, &tmp);
    BinningState bin = carve_binning((char*)binning_buffer, C, &tmp);
    size_t rec_bytes = 0;
    GradRecs recs{}, sums{};
    // the forward recorded the segment length its work list uses (GeomState::fwd_seg_ck); the grid is
    // sized for the shortest segments (seg_ck = 1), so it covers whatever the forward used
    const size_t max_units = R > 0 ? bwd_max_units((size_t)R, tiles, 1) : 0;
    uint32_t *live = nullptr, *live_count = nullptr;
    // the options, each read once
    const int zmode = screen ? 0 : zero_fill_mode();
    const int grid_mode = option(OPT_BWD_GRID);
    // With the outputs zero-filled, gauss_bwd walks a list of the Gaussians with a gradient
    // (~13% of a 1M@1080p view) that gauss_reduce appends to, instead of a lane per Gaussian.
    const bool use_list = zmode != 0 && live_list_mode();
    // atomic backward: per-Gaussian rows (zeroed by the forward, which marked its buffer) instead of records +
    // gauss_reduce; it needs the live list, or a view block (gauss_live_views writes the block's sums and flags);
    // the record path serves every other mode
    const GeomMark mark = geom_marked(geom_buffer);
    const bool atomic = (screen || use_list) && R > 0 && option(OPT_BWD_ATOMIC) != 0 && mark.zeroed;
    // (the atomic backward writes no per-instance records: no record scratch)
    const size_t R_recs = atomic ? 0 : (size_t)R;
    carve_recs(nullptr, R_recs, (size_t)P, &recs, &sums, &live, &live_count, &rec_bytes);
    char* rbase = (char*)call_alloc(scratch_alloc, scratch_ctx, rec_bytes);
    if (!rbase) return fail(GSR_ERR_ALLOC, "rasterize_backward: scratch allocation failed");
    carve_recs(rbase, R_recs, (size_t)P, &recs, &sums, &live, &live_count, &rec_bytes);
    uint32_t* flags = nullptr;
    if (screen) {  // the sums and flags go to the view block (gsr_common.h "View block")
        float* body = view_block + kViewBlockHeader;
        sums.a = reinterpret_cast<float4*>(body);
        sums.b = reinterpret_cast<float4*>(body + 4 * (size_t)P);
        sums.c = reinterpret_cast<float2*>(body + 8 * (size_t)P);
        flags = reinterpret_cast<uint32_t*>(body + 10 * (size_t)P);
    }

    // dense outputs to zero-fill (gauss_bwd then writes only the non-zero rows)
    FillArgs fill{};
    const int m_rest = dc ? M - 1 : M;
    auto seg = [&](float* ptr, size_t n) {
        if (ptr && n) {
            fill.ptr[fill.count] = ptr;
            fill.n[fill.count] = n;
            fill.count++;
        }
    };
    if (zmode) {
        seg(dL_dmean2D, 3 * (size_t)P);
        seg(dL_dconic, 4 * (size_t)P);
        seg(dL_dopacity, (size_t)P);
        seg(dL_dcolor, 3 * (size_t)P);
        seg(dL_dinvdepth, (size_t)P);
        seg(dL_dmean3D, 3 * (size_t)P);
        seg(dL_dcov3D, 6 * (size_t)P);
        if (m_rest > 0) seg(dL_dsh, 3 * (size_t)m_rest * P);
        seg(dc ? dL_ddc : nullptr, 3 * (size_t)P);
        seg(dL_dscale, 3 * (size_t)P);
        seg(dL_drot, 4 * (size_t)P);
    }
    if (!use_list) live = live_count = nullptr;
    if (use_list && R == 0)
        HIP_TRY(hipMemsetAsync(live_count, 0, sizeof(uint32_t) * kLiveShards * kLiveCntStride, stream), "live count");
    SideStream* side = zmode == 1 && !debug && fill.count ? side_stream() : nullptr;
    // Once the fill is queued on the side stream, `stream` must not run ahead of it on ANY return:
    // the caller may free the outputs it writes as soon as this function fails, and the caching
    // allocator would hand their memory to new work on `stream` while the fill still writes it.
    struct SideJoin {
        SideStream* side = nullptr;
        hipStream_t stream = nullptr;
        bool armed = false;
        std::unique_lock<std::mutex> lock;
        void join() {
            if (!armed) return;
            armed = false;
            if (hipStreamWaitEvent(stream, side->join, 0) != hipSuccess) (void)hipStreamSynchronize(side->s);
        }
        ~SideJoin() { join(); }
    } sj;
    if (side) {  // fork: the side stream starts after everything queued so far on `stream`
        sj.lock = std::unique_lock<std::mutex>(side->mu);
        sj.side = side;
        sj.stream = stream;
        HIP_TRY(hipEventRecord(side->fork, stream), "zero fill fork");
        HIP_TRY(hipStreamWaitEvent(side->s, side->fork, 0), "zero fill fork");
        const hipError_t fe = launch_zero_fill(fill, side->s);
        const hipError_t je = hipEventRecord(side->join, side->s);
        if (fe != hipSuccess || je != hipSuccess) {
            (void)hipStreamSynchronize(side->s);  // whatever was queued has finished
            return fail(GSR_ERR_HIP, "zero fill: %s", hipGetErrorString(fe != hipSuccess ? fe : je));
        }
        sj.armed = true;
    }

    // the records' content bytes (zeroed by the forward's K3): render_bwd sets those of the records
    // it writes, gauss_reduce reads them to find the records
    recs.flag = bin.rec_flag;
    // (also with R == 0: gauss_reduce still reads every Gaussian's record start)
    if (!atomic && !mark.recs) {  // a forward that left no record inputs (or a buffer never seen)
        HIP_TRY(launch_rec_prep(P, geom, bin, C, stream), "record prep");
        geom_mark(geom_buffer, mark.zeroed, true, mark.long_lists);
    }
    if (R > 0) {
        StageScope sc(ST_RENDER_BWD, stream);
        RenderBwdArgs ra{};
        ra.W = width; ra.H = height; ra.gx = gx; ra.gy = gy; ra.ranges = img.ranges; ra.gid_sorted = bin.gid_sorted;
        ra.rec = geom.rec;
        ra.bg = background; ra.dL_dpix = dL_dpix; ra.dL_dinvdepth = dL_dinvdepths; ra.img = img; ra.recs = recs;
        ra.ckpt = bin.ckpt; ra.seg_ck = geom.fwd_seg_ck; ra.rec_start = geom.rec_start;
        ra.unit_cnt = geom.unit_cnt; ra.unit_part = geom.unit_part; ra.unit_full = bin.unit_full;
        ra.full_cap = (uint32_t)unit_full_cap(C);
        ra.census = g_census;
        ra.live_count = live_count;  // zeroed by its first workgroup
        if (zmode == 3 && fill.count) {  // the zero fill rides in this launch
            ra.fill = fill;
            ra.fill_blocks = kFusedFillBlocks;
        }
        if (atomic) {
            ra.acc = reinterpret_cast<float*>(geom.acc);
            ra.touched = geom.touched;
        }
        HIP_TRY(launch_render_bwd(ra, max_units, stream, grid_mode), "render_bwd");
    }
    if (int rc = check_debug(debug, stream, "render_bwd")) return rc;
    if (atomic && screen) {  // (stage "gauss_reduce": the step between render_bwd and gauss_bwd / the exchange)
        StageScope sc(ST_GAUSS_REDUCE, stream);
        HIP_TRY(launch_gauss_live_views(P, geom.touched, geom.acc, radii, geom.clamped, sums, flags, stream),
                "gauss_live_views");
    } else if (atomic) {
        // (nothing between render_bwd and gauss_bwd: gauss_bwd lists the touched Gaussians itself)
    } else {
        StageScope sc(ST_GAUSS_REDUCE, stream);
        HIP_TRY(launch_gauss_reduce(P, geom, recs, sums, flags, radii, live, live_count, stream),
                "gauss_reduce");
    }
    if (int rc = check_debug(debug, stream, "gauss_reduce")) return rc;
    if (screen) {
        HIP_TRY(launch_view_header(view_block, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, focal_x, focal_y,
                                   antialiasing, dL_dinvdepths != nullptr, stream),
                "view header");
        return check_debug(debug, stream, "view header");
    }
    {
        StageScope sc(ST_GAUSS_BWD, stream);
        GaussBwdArgs ga{};
        ga.P = P; ga.D = D; ga.M = M; ga.W = width; ga.H = height;
        ga.means3D = means3D; ga.shs = colors_precomp || M <= (dc ? 1 : 0) ? nullptr : shs;
        ga.dc = colors_precomp ? nullptr : dc; ga.opacities = opacities; ga.scales = scales;
        ga.rotations = rotations; ga.cov3D_precomp = cov3D_precomp; ga.scale_modifier = scale_modifier;
        ga.viewmatrix = viewmatrix; ga.projmatrix = projmatrix; ga.campos = campos;
        ga.tan_fovx = tan_fovx; ga.tan_fovy = tan_fovy; ga.focal_x = focal_x; ga.focal_y = focal_y;
        ga.antialiasing = antialiasing; ga.radii = radii; ga.geom = geom; ga.sums = sums;
        ga.have_invdepth = dL_dinvdepths != nullptr;
        ga.dL_dmean2D = dL_dmean2D; ga.dL_dconic = dL_dconic; ga.dL_dopacity = dL_dopacity; ga.dL_dcolor = dL_dcolor;
        ga.dL_dinvdepth = dL_dinvdepth; ga.dL_dmean3D = dL_dmean3D; ga.dL_dcov3D = dL_dcov3D;
        ga.dL_dsh = M > (dc ? 1 : 0) ? dL_dsh : nullptr; ga.dL_ddc = dc ? dL_ddc : nullptr; ga.dL_dscale = dL_dscale; ga.dL_drot = dL_drot;
        if (side) {  // join: gauss_bwd writes over the zeroed outputs
            sj.join();
            sj.lock.unlock();
        } else if (zmode == 1 || zmode == 2 || (zmode == 3 && R == 0)) {  // (3 with R = 0: no render_bwd launch)
            HIP_TRY(launch_zero_fill(fill, stream), "zero fill");
        }
        ga.sparse = zmode ? 1 : 0;
        ga.live = live;
        ga.live_count = live_count;
        ga.live_cap = live_list_cap((uint32_t)P);
        if (atomic) {  // the sums are the accumulator rows of the touched Gaussians (render_bwd ATOMIC)
            ga.touched = geom.touched;
            ga.acc = geom.acc;
            // runs of 128 x N touched-bit positions per workgroup (backward.hip gauss_bwd_touched_kernel): N from
            // the option, or by the frame -- 16 where the lists are long (few Gaussians touched: 5M@4K), else 1
            const int opt_run = option(OPT_TOUCHED_RUN);
            const uint32_t run = opt_run > 0 ? (uint32_t)opt_run : mark.long_lists ? 16u : 1u;
            ga.touched_shift = 31u - (uint32_t)__builtin_clz(run);  // (a power of two at most, floor)
        }
        HIP_TRY(launch_gauss_bwd(ga, stream), "gauss_bwd");
    }
    if (int rc = check_debug(debug, stream, "gauss_bwd")) return rc;
    return GSR_OK;
}
}  // namespace

int gsr_rasterize_backward(int P, int D, int M, int R, const float* background, int width, int height,
                           const float* means3D, const float* shs, const float* colors_precomp,
                           const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                           const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                           const float* campos, float tan_fovx, float tan_fovy, const int* radii, void* geom_buffer,
                           void* binning_buffer, void* image_buffer, const float* dL_dpix, const float* dL_dinvdepths,
                           float* dL_dmean2D, float* dL_dconic, float* dL_dopacity, float* dL_dcolor,
                           float* dL_dinvdepth, float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscale,
                           float* dL_drot, int antialiasing, int debug, gsr_alloc_fn scratch_alloc,
                           void* scratch_ctx, void* stream) {
    return backward_impl(P, D, M, R, background, width, height, means3D, nullptr, shs, colors_precomp, opacities, scales,
                         scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy,
                         radii, geom_buffer, binning_buffer, image_buffer, dL_dpix, dL_dinvdepths, dL_dmean2D,
                         dL_dconic, dL_dopacity, dL_dcolor, dL_dinvdepth, dL_dmean3D, dL_dcov3D, nullptr, dL_dsh, dL_dscale,
                         dL_drot, antialiasing, debug, scratch_alloc, scratch_ctx, stream, 0, 0);
}

int gsr_rasterize_backward_ex(int P, int D, int M, int R, const float* background, int width, int height,
                              const float* means3D, const float* shs, const float* colors_precomp,
                              const float* opacities, const float* scales, float scale_modifier,
                              const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                              const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                              const int* radii, void* geom_buffer, void* binning_buffer, void* image_buffer,
                              const float* dL_dpix, const float* dL_dinvdepths, float* dL_dmean2D, float* dL_dconic,
                              float* dL_dopacity, float* dL_dcolor, float* dL_dinvdepth, float* dL_dmean3D,
                              float* dL_dcov3D, float* dL_dsh, float* dL_dscale, float* dL_drot, int antialiasing,
                              int debug, gsr_alloc_fn scratch_alloc, void* scratch_ctx, void* stream,
                              int binning_capacity, size_t binning_bytes) {
    return backward_impl(P, D, M, R, background, width, height, means3D, nullptr, shs, colors_precomp, opacities, scales,
                         scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy,
                         radii, geom_buffer, binning_buffer, image_buffer, dL_dpix, dL_dinvdepths, dL_dmean2D,
                         dL_dconic, dL_dopacity, dL_dcolor, dL_dinvdepth, dL_dmean3D, dL_dcov3D, nullptr, dL_dsh, dL_dscale,
                         dL_drot, antialiasing, debug, scratch_alloc, scratch_ctx, stream, binning_capacity,
                         binning_bytes);
}

int gsr_rasterize_forward_dc(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                             gsr_alloc_fn image_alloc, void* image_ctx, int P, int D, int M, const float* background,
                             int width, int height, const float* means3D, const float* dc, const float* shs,
                             const float* colors_precomp, const float* opacities, const float* scales,
                             float scale_modifier, const float* rotations, const float* cov3D_precomp,
                             const float* viewmatrix, const float* projmatrix, const float* cam_pos, float tan_fovx,
                             float tan_fovy, int prefiltered, float* out_color, float* out_invdepth, int antialiasing,
                             int* radii, int debug, void* stream, int* num_rendered, int capacity_hint,
                             int* binning_capacity) {
    if (!dc && !colors_precomp)
        return fail(GSR_ERR_ARGUMENT, "rasterize_forward_dc: provide dc (+ shs) or precomputed colours");
    return forward_impl(geom_alloc, geom_ctx, binning_alloc, binning_ctx, image_alloc, image_ctx, P, D, M, background,
                        width, height, means3D, dc, shs, colors_precomp, opacities, scales, scale_modifier, rotations,
                        cov3D_precomp, viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, prefiltered, out_color,
                        out_invdepth, antialiasing, radii, debug, stream, num_rendered, capacity_hint,
                        binning_capacity);
}

int gsr_rasterize_backward_dc(int P, int D, int M, int R, const float* background, int width, int height,
                              const float* means3D, const float* dc, const float* shs, const float* colors_precomp,
                              const float* opacities, const float* scales, float scale_modifier,
                              const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                              const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                              const int* radii, void* geom_buffer, void* binning_buffer, void* image_buffer,
                              const float* dL_dpix, const float* dL_dinvdepths, float* dL_dmean2D, float* dL_dconic,
                              float* dL_dopacity, float* dL_dcolor, float* dL_dinvdepth, float* dL_dmean3D,
                              float* dL_dcov3D, float* dL_ddc, float* dL_dsh, float* dL_dscale, float* dL_drot,
                              int antialiasing, int debug, gsr_alloc_fn scratch_alloc, void* scratch_ctx,
                              void* stream, int binning_capacity, size_t binning_bytes) {
    if (!dc && !colors_precomp)
        return fail(GSR_ERR_ARGUMENT, "rasterize_backward_dc: provide dc (+ shs) or precomputed colours");
    return backward_impl(P, D, M, R, background, width, height, means3D, dc, shs, colors_precomp, opacities, scales,
                         scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy,
                         radii, geom_buffer, binning_buffer, image_buffer, dL_dpix, dL_dinvdepths, dL_dmean2D,
                         dL_dconic, dL_dopacity, dL_dcolor, dL_dinvdepth, dL_dmean3D, dL_dcov3D, dL_ddc, dL_dsh,
                         dL_dscale, dL_drot, antialiasing, debug, scratch_alloc, scratch_ctx, stream,
                         binning_capacity, binning_bytes);
}

}  // extern "C"

// ---- multi-GPU view exchange (include/gsr.h) -----------------------------------------
unsigned long long gsr_view_block_floats(int P) { return P > 0 ? gsr::view_block_floats((size_t)P) : 0ull; }

unsigned long long gsr_view_pack_floats(long long entries) {
    return gsr::view_pack_floats(entries > 0 ? (size_t)entries : 0);
}

unsigned long long gsr_view_pack_scratch_bytes(int P) { return P > 0 ? 4ull * ((P + 255) / 256) : 4ull; }

int gsr_view_block_pack_range(int P, int g0, int g1, const float* view_block, float* packed, long long cap,
                              void* scratch, unsigned int* count, void* stream) {
    g_err[0] = 0;
    if (P <= 0 || cap < 0) return fail(GSR_ERR_ARGUMENT, "view_block_pack: P=%d cap=%lld", P, cap);
    if (g0 < 0 || g1 < g0 || g1 > P) return fail(GSR_ERR_ARGUMENT, "view_block_pack: range [%d, %d) of P=%d", g0, g1, P);
    if (!view_block || !packed || !scratch) return fail(GSR_ERR_ARGUMENT, "view_block_pack: null pointer");
    if ((reinterpret_cast<uintptr_t>(view_block) & 15) || (reinterpret_cast<uintptr_t>(packed) & 15))
        return fail(GSR_ERR_ARGUMENT, "view_block_pack: blocks must be 16-byte aligned");
    HIP_TRY(gsr::launch_view_pack((uint32_t)P, (uint32_t)g0, (uint32_t)g1, view_block, packed, (unsigned long long)cap,
                                  reinterpret_cast<uint32_t*>(scratch), count, (hipStream_t)stream),
            "view_block_pack");
    return GSR_OK;
}

int gsr_view_block_pack(int P, const float* view_block, float* packed, long long cap, void* scratch,
                        unsigned int* count, void* stream) {
    return gsr_view_block_pack_range(P, 0, P, view_block, packed, cap, scratch, count, stream);
}

int gsr_view_block_unpack(int P, int n_views, const float* packed, long long packed_floats, float* blocks,
                          long long cap, void* stream) {
    g_err[0] = 0;
    if (P <= 0 || n_views < 0 || cap < 0 || packed_floats < (long long)gsr::view_pack_floats(0))
        return fail(GSR_ERR_ARGUMENT, "view_block_unpack: P=%d views=%d packed_floats=%lld cap=%lld", P, n_views,
                    packed_floats, cap);
    if ((size_t)packed_floats < gsr::view_pack_floats((size_t)cap))
        return fail(GSR_ERR_ARGUMENT, "view_block_unpack: %lld floats per packed block cannot hold %lld entries",
                    packed_floats, cap);
    if (n_views > 0 && (!packed || !blocks)) return fail(GSR_ERR_ARGUMENT, "view_block_unpack: null pointer");
    if ((reinterpret_cast<uintptr_t>(packed) & 15) || (reinterpret_cast<uintptr_t>(blocks) & 15) || (packed_floats & 3))
        return fail(GSR_ERR_ARGUMENT, "view_block_unpack: blocks must be 16-byte aligned");
    HIP_TRY(gsr::launch_view_unpack((uint32_t)P, n_views, packed, (unsigned long long)packed_floats, blocks,
                                    (unsigned long long)cap, (hipStream_t)stream),
            "view_block_unpack");
    return GSR_OK;
}

int gsr_view_block_index(int P, int n_views, const float* packed, long long packed_floats, unsigned int* flags,
                         long long cap, void* stream) {
    return gsr_view_block_index_range(P, 0, P, n_views, packed, packed_floats, flags, cap, stream);
}

int gsr_view_block_index_range(int P, int g0, int g1, int n_views, const float* packed, long long packed_floats,
                               unsigned int* flags, long long cap, void* stream) {
    g_err[0] = 0;
    if (g0 < 0 || g1 < g0 || g1 > P) return fail(GSR_ERR_ARGUMENT, "view_block_index: range [%d, %d) of P=%d", g0, g1, P);
    if (P <= 0 || n_views < 0 || cap < 0 || packed_floats < (long long)gsr::view_pack_floats(0))
        return fail(GSR_ERR_ARGUMENT, "view_block_index: P=%d views=%d packed_floats=%lld cap=%lld", P, n_views,
                    packed_floats, cap);
    if ((size_t)packed_floats < gsr::view_pack_floats((size_t)cap))
        return fail(GSR_ERR_ARGUMENT, "view_block_index: %lld floats per packed block cannot hold %lld entries",
                    packed_floats, cap);
    if (cap >= (1ll << 28)) return fail(GSR_ERR_ARGUMENT, "view_block_index: %lld entries exceed 2^28", cap);
    if (n_views > 0 && (!packed || !flags)) return fail(GSR_ERR_ARGUMENT, "view_block_index: null pointer");
    if ((reinterpret_cast<uintptr_t>(packed) & 15) || (packed_floats & 3))
        return fail(GSR_ERR_ARGUMENT, "view_block_index: packed blocks must be 16-byte aligned");
    HIP_TRY(gsr::launch_view_index((uint32_t)P, (uint32_t)g0, (uint32_t)g1, n_views, packed,
                                   (unsigned long long)packed_floats, flags, (unsigned long long)cap, (hipStream_t)stream),
            "view_block_index");
    return GSR_OK;
}

int gsr_rasterize_backward_screen(int P, int D, int M, int R, const float* background, int width, int height,
                                  const float* means3D, const float* dc, const float* shs, const float* opacities,
                                  const float* scales, float scale_modifier, const float* rotations,
                                  const float* viewmatrix, const float* projmatrix, const float* campos,
                                  float tan_fovx, float tan_fovy, const int* radii, void* geom_buffer,
                                  void* binning_buffer, void* image_buffer, const float* dL_dpix,
                                  const float* dL_dinvdepths, int antialiasing, int debug, gsr_alloc_fn scratch_alloc,
                                  void* scratch_ctx, void* stream, int binning_capacity, size_t binning_bytes,
                                  float* view_block) {
    if (!view_block) return fail(GSR_ERR_ARGUMENT, "rasterize_backward_screen: null view block");
    if ((reinterpret_cast<uintptr_t>(view_block) & 15) != 0)
        return fail(GSR_ERR_ARGUMENT, "rasterize_backward_screen: view block must be 16-byte aligned");
    return backward_impl(P, D, M, R, background, width, height, means3D, dc, shs, nullptr, opacities, scales,
                         scale_modifier, rotations, nullptr, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, radii,
                         geom_buffer, binning_buffer, image_buffer, dL_dpix, dL_dinvdepths, nullptr, nullptr, nullptr,
                         nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, antialiasing, debug,
                         scratch_alloc, scratch_ctx, stream, binning_capacity, binning_bytes, view_block);
}

int gsr_debug_forward_state(int P, int width, int height, int R, int binning_capacity, size_t binning_bytes,
                            const void* geom_buffer, const void* binning_buffer, const void* image_buffer,
                            unsigned int* ranges, unsigned int* point_list, unsigned int* n_contrib, float* final_T,
                            void* stream_) {
    using namespace gsr;
    g_err[0] = 0;
    hipStream_t stream = (hipStream_t)stream_;
    if (P <= 0 || R < 0 || width <= 0 || height <= 0)
        return fail(GSR_ERR_ARGUMENT, "debug_forward_state: invalid sizes P=%d R=%d W=%d H=%d", P, R, width, height);
    if (!image_buffer || (R > 0 && !binning_buffer))
        return fail(GSR_ERR_ARGUMENT, "debug_forward_state: missing forward buffers");
    size_t C = 0, tmp = 0;
    if (!resolve_capacity(R, binning_capacity, binning_bytes, &C) || C < (size_t)R)
        return fail(GSR_ERR_ARGUMENT, "debug_forward_state: binning buffer of %zu bytes matches no layout for R=%d",
                    binning_bytes, R);
    const uint32_t gx = (width + kTile - 1) / kTile, gy = (height + kTile - 1) / kTile;
    ImageState img = carve_image((char*)image_buffer, width, height, gx * gy, &tmp);
    const size_t N = (size_t)width * height;
    if (ranges) HIP_TRY(hipMemcpyAsync(ranges, img.ranges, sizeof(uint2) * gx * gy, hipMemcpyDeviceToDevice, stream),
                        "debug_forward_state ranges");
    (void)N;
    if (n_contrib)
        HIP_TRY(launch_untile(img.n_contrib, n_contrib, width, height, gx, stream), "debug_forward_state n_contrib");
    if (final_T)
        HIP_TRY(launch_untile(reinterpret_cast<const uint32_t*>(img.final_T), reinterpret_cast<uint32_t*>(final_T),
                              width, height, gx, stream),
                "debug_forward_state final_T");
    if (point_list && R > 0) {
        // the forward's sorted entries (masks included) and, where K4 sorted only a list's reachable
        // prefix, the rest of the list sorted here into the copy
        if (!geom_buffer) return fail(GSR_ERR_ARGUMENT, "debug_forward_state: point_list needs the geometry buffer");
        BinningState bin = carve_binning((char*)binning_buffer, C, &tmp);
        GeomState geom = carve_geom((char*)const_cast<void*>(geom_buffer), P, gx, gy, &tmp);
        HIP_TRY(launch_sorted_lists_copy(gx * gy, img.ranges, geom, bin, C, point_list, stream, P, gx, true),
                "debug_forward_state point_list");
    }
    return GSR_OK;
}

int gsr_debug_sort_state(int P, int width, int height, const void* geom_buffer, unsigned int* sorted_len,
                         unsigned int* redo_count, void* stream_) {
    using namespace gsr;
    g_err[0] = 0;
    hipStream_t stream = (hipStream_t)stream_;
    if (P <= 0 || width <= 0 || height <= 0 || !geom_buffer)
        return fail(GSR_ERR_ARGUMENT, "debug_sort_state: invalid sizes or no geometry buffer");
    const uint32_t gx = (width + kTile - 1) / kTile, gy = (height + kTile - 1) / kTile;
    size_t tmp = 0;
    GeomState geom = carve_geom((char*)const_cast<void*>(geom_buffer), P, gx, gy, &tmp);
    if (sorted_len)
        HIP_TRY(hipMemcpyAsync(sorted_len, geom.sorted_len, sizeof(uint32_t) * gx * gy, hipMemcpyDeviceToDevice, stream),
                "debug_sort_state sorted_len");
    if (redo_count)
        HIP_TRY(hipMemcpyAsync(redo_count, geom.redo_cnt, sizeof(uint32_t), hipMemcpyDeviceToDevice, stream),
                "debug_sort_state redo_count");
    return GSR_OK;
}

int gsr_debug_near_state(int P, int width, int height, const void* geom_buffer, unsigned int* zcut,
                         unsigned int* near_ranges, void* stream_) {
    using namespace gsr;
    g_err[0] = 0;
    hipStream_t stream = (hipStream_t)stream_;
    if (P <= 0 || width <= 0 || height <= 0 || !geom_buffer)
        return fail(GSR_ERR_ARGUMENT, "debug_near_state: invalid sizes or no geometry buffer");
    const uint32_t gx = (width + kTile - 1) / kTile, gy = (height + kTile - 1) / kTile;
    size_t tmp = 0;
    GeomState geom = carve_geom((char*)const_cast<void*>(geom_buffer), P, gx, gy, &tmp);
    if (zcut)
        HIP_TRY(hipMemcpyAsync(zcut, geom.zcut, sizeof(uint32_t), hipMemcpyDeviceToDevice, stream), "debug_near_state zcut");
    if (near_ranges)
        HIP_TRY(hipMemcpyAsync(near_ranges, geom.sranges, sizeof(uint2) * gx * gy, hipMemcpyDeviceToDevice, stream),
                "debug_near_state sranges");
    return GSR_OK;
}

namespace {
int backward_views_impl(int P, int D, int M, const float* means3D, const float* dc, const float* shs,
                        const float* opacities, const float* scales, const float* rotations, float scale_modifier,
                        int n_views, const float* blocks, long long block_floats, const unsigned int* flags,
                        const unsigned int* live, const unsigned int* live_count, float* dL_dmean3D, float* dL_ddc,
                        float* dL_dsh, float* dL_dopacity, float* dL_dscale, float* dL_drot, void* stream) {
    using namespace gsr;
    g_err[0] = 0;
    if (P < 0 || n_views < 0) return fail(GSR_ERR_ARGUMENT, "gauss_backward_views: P=%d views=%d", P, n_views);
    if (P == 0) return GSR_OK;
    if (!flags && (size_t)block_floats != view_block_floats((size_t)P))
        return fail(GSR_ERR_ARGUMENT, "gauss_backward_views: block of %lld floats, expected %zu", block_floats,
                    view_block_floats((size_t)P));
    if (flags && (block_floats < (long long)view_pack_floats(0) || (block_floats & 3) ||
                  (reinterpret_cast<uintptr_t>(blocks) & 15)))
        return fail(GSR_ERR_ARGUMENT, "gauss_backward_views: packed blocks of %lld floats (16-byte aligned)",
                    block_floats);
    if (!means3D || !opacities || !scales || !rotations || (n_views > 0 && !blocks) || !dL_dmean3D || !dL_dopacity ||
        !dL_dscale || !dL_drot)
        return fail(GSR_ERR_ARGUMENT, "gauss_backward_views: null pointer");
    if (D < 0 || D > 3) return fail(GSR_ERR_ARGUMENT, "gauss_backward_views: SH degree %d", D);
    if (dc && M > 0 && !shs) return fail(GSR_ERR_ARGUMENT, "gauss_backward_views: rest SH without shs");
    if ((shs && !dL_dsh) || (dc && !dL_ddc)) return fail(GSR_ERR_ARGUMENT, "gauss_backward_views: missing SH outputs");
    if (!dc && !shs) return fail(GSR_ERR_ARGUMENT, "gauss_backward_views: needs SH (precomputed colours are per view)");
    if ((D + 1) * (D + 1) > (dc ? M + 1 : M))  // as the forward (forward_impl): never read past a row
        return fail(GSR_ERR_ARGUMENT, "gauss_backward_views: SH degree %d needs %d coefficients, got %d", D,
                    (D + 1) * (D + 1), dc ? M + 1 : M);
    ViewsBwdArgs a{};
    a.P = P; a.D = D; a.M = dc ? M + 1 : M;
    a.means3D = means3D; a.shs = (dc && M == 0) ? nullptr : shs; a.dc = dc; a.opacities = opacities; a.scales = scales;
    a.rotations = rotations; a.scale_modifier = scale_modifier; a.n_views = n_views; a.blocks = blocks;
    a.block_floats = (size_t)block_floats;
    a.flags = flags;
    a.live = live;
    a.live_count = live_count;
    a.live_cap = live_list_cap((uint32_t)P);
    a.dL_dmean3D = dL_dmean3D; a.dL_dsh = a.shs ? dL_dsh : nullptr; a.dL_ddc = dc ? dL_ddc : nullptr;
    a.dL_dopacity = dL_dopacity; a.dL_dscale = dL_dscale; a.dL_drot = dL_drot;
    {
        StageScope sc(ST_GAUSS_BWD, (hipStream_t)stream);
        HIP_TRY(launch_gauss_bwd_views(a, (hipStream_t)stream), "gauss_backward_views");
    }
    return GSR_OK;
}
}  // namespace

int gsr_gauss_backward_views(int P, int D, int M, const float* means3D, const float* dc, const float* shs,
                             const float* opacities, const float* scales, const float* rotations, float scale_modifier,
                             int n_views, const float* blocks, long long block_floats, float* dL_dmean3D,
                             float* dL_ddc, float* dL_dsh, float* dL_dopacity, float* dL_dscale, float* dL_drot,
                             void* stream) {
    return backward_views_impl(P, D, M, means3D, dc, shs, opacities, scales, rotations, scale_modifier, n_views,
                               blocks, block_floats, nullptr, nullptr, nullptr, dL_dmean3D, dL_ddc, dL_dsh, dL_dopacity,
                               dL_dscale, dL_drot, stream);
}

int gsr_gauss_backward_views_packed(int P, int D, int M, const float* means3D, const float* dc, const float* shs,
                                    const float* opacities, const float* scales, const float* rotations,
                                    float scale_modifier, int n_views, const float* packed, long long packed_floats,
                                    const unsigned int* flags, float* dL_dmean3D, float* dL_ddc, float* dL_dsh,
                                    float* dL_dopacity, float* dL_dscale, float* dL_drot, void* stream) {
    if (n_views > 0 && !flags) return fail(GSR_ERR_ARGUMENT, "gauss_backward_views_packed: null flags");
    return backward_views_impl(P, D, M, means3D, dc, shs, opacities, scales, rotations, scale_modifier, n_views,
                               packed, packed_floats, flags, nullptr, nullptr, dL_dmean3D, dL_ddc, dL_dsh, dL_dopacity,
                               dL_dscale, dL_drot, stream);
}

unsigned long long gsr_views_live_floats(int P) {
    return P > 0 ? (unsigned long long)gsr::kLiveShards * gsr::live_list_cap((uint32_t)P) +
                       (unsigned long long)gsr::kLiveShards * gsr::kLiveCntStride
                 : 0ull;
}

int gsr_views_live_list_range(int P, int g0, int g1, int n_views, const unsigned int* flags, unsigned int* live,
                              void* stream) {
    g_err[0] = 0;
    if (P < 0 || n_views < 0) return fail(GSR_ERR_ARGUMENT, "views_live_list: P=%d views=%d", P, n_views);
    if (g0 < 0 || g1 < g0 || g1 > P) return fail(GSR_ERR_ARGUMENT, "views_live_list: range [%d, %d) of P=%d", g0, g1, P);
    if (P == 0) return GSR_OK;
    if (!live || (n_views > 0 && !flags)) return fail(GSR_ERR_ARGUMENT, "views_live_list: null pointer");
    unsigned int* count = live + (size_t)gsr::kLiveShards * gsr::live_list_cap((uint32_t)P);
    HIP_TRY(gsr::launch_views_live((uint32_t)P, (uint32_t)g0, (uint32_t)g1, n_views, flags, live, count,
                                   (hipStream_t)stream),
            "views_live_list");
    return GSR_OK;
}

int gsr_views_live_list(int P, int n_views, const unsigned int* flags, unsigned int* live, void* stream) {
    return gsr_views_live_list_range(P, 0, P, n_views, flags, live, stream);
}

int gsr_gauss_backward_views_live(int P, int D, int M, const float* means3D, const float* dc, const float* shs,
                                  const float* opacities, const float* scales, const float* rotations,
                                  float scale_modifier, int n_views, const float* packed, long long packed_floats,
                                  const unsigned int* flags, const unsigned int* live, float* dL_dmean3D,
                                  float* dL_ddc, float* dL_dsh, float* dL_dopacity, float* dL_dscale, float* dL_drot,
                                  void* stream) {
    if (n_views > 0 && (!flags || !live)) return fail(GSR_ERR_ARGUMENT, "gauss_backward_views_live: null list");
    const unsigned int* count = live ? live + (size_t)gsr::kLiveShards * gsr::live_list_cap((uint32_t)(P > 0 ? P : 0))
                                     : nullptr;
    return backward_views_impl(P, D, M, means3D, dc, shs, opacities, scales, rotations, scale_modifier, n_views,
                               packed, packed_floats, flags, live, count, dL_dmean3D, dL_ddc, dL_dsh, dL_dopacity,
                               dL_dscale, dL_drot, stream);
}
