// gpuhash.cpp -- C-ABI host library: contexts, per-device streams, static sharding,
// launch sequencing and the host argmin.  See include/gpuhash.h for the contract and
// the reference call sites it replaces.
#include "gpuhash.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "kernels.h"
#include "plan.h"

using namespace gpuhash;

namespace {

// Nonces per device in one slice of a search (gpuhash_min_ex): 2^38 is ~8 s of work on
// one MI355X at config-2 rates.
constexpr uint64_t kSlicePerDevice = 1ull << 38;

// Per kernel-variant group in the launch metadata: the work counter, then the 4 clock words
// the scan kernel writes (start/end s_memtime and s_memrealtime of workgroup 0).
constexpr size_t kCounterBytes = 40;

struct Dev {
    int ord = -1;
    int shard = -1;        // position in gpuhash_open's device list
    int stream_dev = -1;   // ordinal the runtime reports for `stream` (hipStreamGetDevice)
    hipStream_t stream = nullptr;
    unsigned long long* d_thresh = nullptr;
    Cand* d_cands = nullptr;
    unsigned int* d_ncand = nullptr;
    Cand* d_best = nullptr;
    Cand* h_best = nullptr;  // pinned
    uint32_t cap = 0;
    // launch descriptors + prefix offsets + per-launch work counters, staged through a
    // pinned host buffer and copied once per call
    uint8_t* d_meta = nullptr;
    uint8_t* h_meta = nullptr;
    size_t meta_cap = 0;
    // uniform K+W tables of C2/J=0 descriptors (one per digit count), grow-only
    uint32_t* d_ktab = nullptr;
    size_t ktab_cap = 0;  // words
    // pinned copy of the per-group work counters + clock samples (kCounterBytes each)
    unsigned long long* h_clk = nullptr;
    size_t clk_cap = 0;  // groups
    std::vector<hipEvent_t> ev;
    hipEvent_t done = nullptr;  // blocking-sync event: the end of a call's work (host_wait)
    int wait_mode = 0;          // HostWait
    // per-call results
    int rc = GPUHASH_OK;
    uint64_t best_h = ~0ull, best_n = ~0ull;
    bool used = false;
    double kernel_ms = 0;
    uint32_t launches = 0;
    std::vector<gpuhash_launch_record> recs;
};

}  // namespace

struct gpuhash_ctx {
    // One search at a time per context (a miner runs one job at a time, p1.pdf p.13);
    // concurrent callers, e.g. several goroutines sharing an Engine, are serialised here.
    std::mutex mu;
    std::vector<Dev> devs;
    int policy = kLayoutAuto;
    gpuhash_stats last{};
    std::vector<gpuhash_launch_record> recs;
};

// Restores the calling thread's current HIP device on scope exit.  The ABI runs device
// work on the caller's thread for single-device contexts, and a host sharing that thread
// (a cgo-locked goroutine, a torch process on another device) must not find its current
// device changed by a gpuhash call.
struct DeviceGuard {
    int prev = -1;
    DeviceGuard() {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    }
    ~DeviceGuard() {
        if (prev >= 0) hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

#define HIPCHK(expr)                                \
    do {                                            \
        if ((expr) != hipSuccess) return GPUHASH_EHIP; \
    } while (0)

// How the host waits for a call's work (GPUHASH_HOST_WAIT, read at gpuhash_open):
//   poll    (default) hipEventQuery on a completion event: back to back for the first
//           0.5 ms (short calls return at once), then every 100 us with the thread asleep
//   stream  hipStreamSynchronize on the device's stream
//   event   hipEventSynchronize on the event, created with hipEventBlockingSync
// A miner spends almost all its life inside this wait (a 2^34-nonce job is ~0.5 s of GPU
// time, ~4 s with 8 miners on one GPU).  On this ROCm both `stream` and `event` keep the
// waiting thread running: 8 miners sharing one MI355X burned 1.0 host core each (8 of the
// box's 16-CPU quota), `poll` 0.007 core each, at the same GPU throughput and the same
// bench GH/s (tools/host_wait_probe.py, profiles/r05_host_wait.jsonl).
enum HostWait { kWaitPoll = 0, kWaitStream = 1, kWaitEvent = 2 };

static int host_wait_mode() {
    const char* e = std::getenv("GPUHASH_HOST_WAIT");
    if (e && !std::strcmp(e, "stream")) return kWaitStream;
    if (e && !std::strcmp(e, "event")) return kWaitEvent;
    return kWaitPoll;
}

static int host_wait(Dev& d) {
    if (d.wait_mode == kWaitStream) {
        HIPCHK(hipStreamSynchronize(d.stream));
        return GPUHASH_OK;
    }
    HIPCHK(hipEventRecord(d.done, d.stream));
    if (d.wait_mode == kWaitEvent) {
        HIPCHK(hipEventSynchronize(d.done));
        return GPUHASH_OK;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t q = hipEventQuery(d.done);
        if (q == hipSuccess) return GPUHASH_OK;
        if (q != hipErrorNotReady) return GPUHASH_EHIP;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(500))
            std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
}

static int dev_init(Dev& d, int ord, int shard) {
    d.ord = ord;
    d.shard = shard;
    DeviceGuard guard;
    HIPCHK(hipSetDevice(ord));
    HIPCHK(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    hipDevice_t sd = -1;
    HIPCHK(hipStreamGetDevice(d.stream, &sd));
    if (sd != ord) return GPUHASH_EHIP;  // the stream must live on the device it serves
    d.stream_dev = sd;
    d.wait_mode = host_wait_mode();
    HIPCHK(hipEventCreateWithFlags(&d.done, hipEventBlockingSync | hipEventDisableTiming));
    if (hipMalloc(&d.d_thresh, sizeof(unsigned long long)) != hipSuccess) return GPUHASH_ENOMEM;
    if (hipMalloc(&d.d_ncand, sizeof(unsigned int)) != hipSuccess) return GPUHASH_ENOMEM;
    if (hipMalloc(&d.d_best, sizeof(Cand)) != hipSuccess) return GPUHASH_ENOMEM;
    if (hipHostMalloc(&d.h_best, sizeof(Cand), hipHostMallocDefault) != hipSuccess) return GPUHASH_ENOMEM;
    HIPCHK(hipMemset(d.d_ncand, 0, sizeof(unsigned int)));
    return GPUHASH_OK;
}

static void dev_free(Dev& d) {
    if (d.ord < 0) return;
    DeviceGuard guard;
    hipSetDevice(d.ord);
    if (d.stream) hipStreamSynchronize(d.stream);
    for (auto e : d.ev) hipEventDestroy(e);
    d.ev.clear();
    if (d.done) hipEventDestroy(d.done);
    if (d.d_thresh) hipFree(d.d_thresh);
    if (d.d_ncand) hipFree(d.d_ncand);
    if (d.d_best) hipFree(d.d_best);
    if (d.d_cands) hipFree(d.d_cands);
    if (d.h_best) hipHostFree(d.h_best);
    if (d.d_meta) hipFree(d.d_meta);
    if (d.d_ktab) hipFree(d.d_ktab);
    if (d.h_clk) hipHostFree(d.h_clk);
    if (d.h_meta) hipHostFree(d.h_meta);
    if (d.stream) hipStreamDestroy(d.stream);
    d = Dev{};
}

static int dev_reserve_meta(Dev& d, size_t bytes) {
    if (bytes <= d.meta_cap) return GPUHASH_OK;
    if (d.d_meta) hipFree(d.d_meta);
    if (d.h_meta) hipHostFree(d.h_meta);
    d.d_meta = nullptr;
    d.h_meta = nullptr;
    d.meta_cap = 0;
    size_t cap = std::max<size_t>(bytes, 64 * 1024);
    if (hipMalloc(&d.d_meta, cap) != hipSuccess) return GPUHASH_ENOMEM;
    if (hipHostMalloc(&d.h_meta, cap, hipHostMallocDefault) != hipSuccess) return GPUHASH_ENOMEM;
    d.meta_cap = cap;
    return GPUHASH_OK;
}

static int dev_reserve_ktab(Dev& d, size_t words) {
    if (words <= d.ktab_cap) return GPUHASH_OK;
    if (d.d_ktab) hipFree(d.d_ktab);
    d.d_ktab = nullptr;
    d.ktab_cap = 0;
    if (hipMalloc(&d.d_ktab, words * sizeof(uint32_t)) != hipSuccess) return GPUHASH_ENOMEM;
    d.ktab_cap = words;
    return GPUHASH_OK;
}

static int dev_reserve_clk(Dev& d, size_t groups) {
    if (groups <= d.clk_cap) return GPUHASH_OK;
    if (d.h_clk) hipHostFree(d.h_clk);
    d.h_clk = nullptr;
    d.clk_cap = 0;
    const size_t n = std::max<size_t>(groups, 8);
    if (hipHostMalloc(&d.h_clk, kCounterBytes * n, hipHostMallocDefault) != hipSuccess) return GPUHASH_ENOMEM;
    d.clk_cap = n;
    return GPUHASH_OK;
}

static int dev_reserve(Dev& d, uint32_t cap, size_t nev) {
    if (cap > d.cap) {
        if (d.d_cands) hipFree(d.d_cands);
        d.d_cands = nullptr;
        d.cap = 0;
        if (hipMalloc(&d.d_cands, (size_t)cap * sizeof(Cand)) != hipSuccess) return GPUHASH_ENOMEM;
        d.cap = cap;
    }
    while (d.ev.size() < nev) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        d.ev.push_back(e);
    }
    return GPUHASH_OK;
}

// Runs one device's shard.  The planned launches are grouped by kernel variant; each
// group is ONE persistent launch over all its descriptors (guided self-scheduling, see
// scan_kernel.h), followed by the candidate reduce.  One 16-byte copy back at the end.
// mode 1 writes per-nonce hashes to d_dump instead.
static int dev_run(Dev& d, const uint8_t* msg, size_t len, uint64_t lo, uint64_t hi,
                   uint32_t rchunk, int mode, unsigned long long* d_dump, int policy) {
    d.used = true;
    d.kernel_ms = 0;
    d.launches = 0;
    d.recs.clear();
    DeviceGuard guard;
    HIPCHK(hipSetDevice(d.ord));
    std::vector<Launch> plan;
    plan_range(msg, len, lo, hi, plan, rchunk, policy);

    struct Group {
        int J, C2, EX;
        std::vector<size_t> idx;
    };
    std::vector<Group> groups;
    for (size_t i = 0; i < plan.size(); i++) {
        const Launch& l = plan[i];
        auto it = std::find_if(groups.begin(), groups.end(), [&](const Group& g) {
            return g.J == l.J && g.C2 == l.C2 && g.EX == l.EX;
        });
        if (it == groups.end()) {
            groups.push_back(Group{l.J, l.C2, l.EX, {}});
            it = groups.end() - 1;
        }
        it->idx.push_back(i);
    }

    // meta layout: [per group: work counter + 4 clock words, 40 B][per group: offs
    // (n+1) x 8 B, descs, and for C2 = 3 the launches' p-tables]
    size_t bytes = kCounterBytes * groups.size();
    std::vector<size_t> offs_at(groups.size()), desc_at(groups.size()), ptab_at(groups.size());
    for (size_t g = 0; g < groups.size(); g++) {
        offs_at[g] = bytes;
        bytes += 8 * (groups[g].idx.size() + 1);
        bytes = (bytes + 15) & ~(size_t)15;
        desc_at[g] = bytes;
        bytes += sizeof(LaunchDesc) * groups[g].idx.size();
        bytes = (bytes + 15) & ~(size_t)15;
        ptab_at[g] = bytes;
        for (size_t k : groups[g].idx) bytes += sizeof(uint32_t) * plan[k].nptab;
        bytes = (bytes + 15) & ~(size_t)15;
    }
    int rc = dev_reserve_meta(d, bytes);
    if (rc) return rc;
    std::memset(d.h_meta, 0, kCounterBytes * groups.size());
    std::vector<unsigned int> grids(groups.size());
    // C2/J=0 tables: block B's words depend only on the digit count d, so one table per
    // d serves every descriptor of that digit group; built by k_ktab from the device
    // copy of the first such descriptor (at desc_at[g] + k * sizeof(LaunchDesc)).
    struct Tab { int d; uint32_t off, R; size_t desc_byte; };
    std::vector<Tab> tabs;
    size_t tab_words = 0;
    for (size_t g = 0; g < groups.size(); g++) {
        auto* offs = reinterpret_cast<unsigned long long*>(d.h_meta + offs_at[g]);
        auto* descs = reinterpret_cast<LaunchDesc*>(d.h_meta + desc_at[g]);
        uint32_t ptab_words = 0;
        unsigned long long acc = 0;
        for (size_t k = 0; k < groups[g].idx.size(); k++) {
            const Launch& l = plan[groups[g].idx[k]];
            const LaunchDesc& D = l.desc;
            offs[k] = acc;
            acc += (unsigned long long)((D.p_last - D.p_first) / (uint32_t)kBlock + 1u) * D.R;
            descs[k] = D;
            if (l.C2 == 3) {  // lane table: room for this launch's p-table (k_ptab fills it)
                descs[k].tab_off = ptab_words;
                ptab_words += l.nptab;
            }
            if (l.C2 == 1 && l.J == 0) {
                auto it = std::find_if(tabs.begin(), tabs.end(), [&](const Tab& t) { return t.d == l.d; });
                if (it == tabs.end()) {
                    tabs.push_back(Tab{l.d, (uint32_t)tab_words, D.R, desc_at[g] + k * sizeof(LaunchDesc)});
                    tab_words += 64ull * D.R;
                    it = tabs.end() - 1;
                }
                descs[k].tab_off = it->off;
            }
        }
        offs[groups[g].idx.size()] = acc;
        unsigned int full = grid_for(groups[g].J, groups[g].C2, groups[g].EX, mode, d.ord);
        if (full == 0) return GPUHASH_EHIP;
        // no more workgroups than minimum-size pieces
        unsigned long long pieces = (acc + 9) / 10;
        grids[g] = (unsigned int)std::min<unsigned long long>(full, std::max<unsigned long long>(pieces, 1));
    }
    // every workgroup of every group may append one candidate before the single reduce
    uint32_t sumgrid = 0;
    for (unsigned int gr : grids) sumgrid += gr;
    rc = dev_reserve(d, std::max<uint32_t>(sumgrid, 1u), 2 * groups.size());
    if (rc) return rc;
    if (tab_words && (rc = dev_reserve_ktab(d, tab_words))) return rc;
    if ((rc = dev_reserve_clk(d, groups.size()))) return rc;
    HIPCHK(hipMemcpyAsync(d.d_meta, d.h_meta, bytes, hipMemcpyHostToDevice, d.stream));
    for (const Tab& t : tabs)
        HIPCHK(launch_ktab(reinterpret_cast<const LaunchDesc*>(d.d_meta + t.desc_byte), d.d_ktab + t.off,
                           t.R, d.stream));
    // lane-table groups: their launches' p-tables, one device thread per block B-1 value
    // (on the host these compressions cost ~0.16 us each, ~7% of a search whose loop
    // values cover only 10^5 lane values each)
    for (size_t g = 0; g < groups.size(); g++)
        if (groups[g].C2 == 3)
            HIPCHK(launch_ptab(reinterpret_cast<const LaunchDesc*>(d.d_meta + desc_at[g]),
                               (int)groups[g].idx.size(), reinterpret_cast<uint32_t*>(d.d_meta + ptab_at[g]),
                               d.stream));
    HIPCHK(hipMemsetAsync(d.d_thresh, 0xFF, sizeof(unsigned long long), d.stream));
    HIPCHK(hipMemsetAsync(d.d_best, 0xFF, sizeof(Cand), d.stream));
    HIPCHK(hipMemsetAsync(d.d_ncand, 0, sizeof(unsigned int), d.stream));
    const unsigned int gmax = rchunk ? rchunk : 400u;
    const unsigned int gmin = std::min(10u, gmax);
    // Groups run back to back on the device's stream (each launch's HIP events then time
    // that kernel alone, which bench.py's roofline relies on).  Running the small groups
    // on a second stream was measured: a persistent grid launched beside another is not
    // fully dispatched until the other drains, so its events span the whole call, for
    // <= 0.3% less wall time.  All groups append to one candidate list (atomic counter,
    // shared pruning threshold); one reduce at the end folds it.
    for (size_t g = 0; g < groups.size(); g++) {
        ScanArgs a{};
        a.stream = d.stream;
        a.descs = reinterpret_cast<const LaunchDesc*>(d.d_meta + desc_at[g]);
        a.offs = reinterpret_cast<const unsigned long long*>(d.d_meta + offs_at[g]);
        a.ndesc = (int)groups[g].idx.size();
        a.work = reinterpret_cast<unsigned long long*>(d.d_meta + kCounterBytes * g);
        a.gmin = gmin;
        a.gmax = gmax;
        a.thresh = d.d_thresh;
        a.cands = d.d_cands;
        a.ncand = d.d_ncand;
        a.dump = d_dump;
        a.dump_lo = lo;
        a.ktab = groups[g].C2 == 3 ? reinterpret_cast<const uint32_t*>(d.d_meta + ptab_at[g]) : d.d_ktab;
        a.grid = grids[g];
        HIPCHK(hipEventRecord(d.ev[2 * g], a.stream));
        HIPCHK(launch_scan(groups[g].J, groups[g].C2, groups[g].EX, mode, a));
        HIPCHK(hipEventRecord(d.ev[2 * g + 1], a.stream));
    }
    if (mode == 0) HIPCHK(launch_reduce(d.d_cands, d.d_ncand, d.d_best, d.stream));
    HIPCHK(hipMemcpyAsync(d.h_best, d.d_best, sizeof(Cand), hipMemcpyDeviceToHost, d.stream));
    HIPCHK(hipMemcpyAsync(d.h_clk, d.d_meta, kCounterBytes * groups.size(), hipMemcpyDeviceToHost, d.stream));
    if ((rc = host_wait(d))) return rc;
    for (size_t g = 0; g < groups.size(); g++) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, d.ev[2 * g], d.ev[2 * g + 1]));
        d.kernel_ms += ms;
        uint64_t nonces = 0, biggest = 0;
        const Launch* big = nullptr;
        for (size_t k : groups[g].idx) {
            const Launch& l = plan[k];
            uint64_t n = (l.hi - l.lo) / l.stride + 1;
            nonces += n;
            if (!big || n > biggest) { big = &l; biggest = n; }
        }
        const unsigned long long* c = d.h_clk + (kCounterBytes / 8) * g + 1;
        const double ticks = (double)(c[2] - c[0]), rt = (double)(c[3] - c[1]);
        const double sclk = rt > 0 ? ticks / rt * 100.0 : 0.0;  // s_memrealtime runs at 100 MHz
        d.recs.push_back(gpuhash_launch_record{d.ord, groups[g].J, groups[g].C2, groups[g].EX,
                                               big->d, big->c, d.shard, d.stream_dev, lo, hi,
                                               nonces, (double)ms, sclk});
    }
    d.launches = (uint32_t)groups.size();
    d.best_h = d.h_best->hash;
    d.best_n = d.h_best->nonce;
    return GPUHASH_OK;
}

extern "C" {

static int open_impl(const int* devices, int ndevices, gpuhash_ctx** out);

int gpuhash_open(const int* devices, int ndevices, gpuhash_ctx** out) {
    if (!out || ndevices < 0 || (ndevices > 0 && !devices)) return GPUHASH_EINVAL;
    *out = nullptr;
    try {
        return open_impl(devices, ndevices, out);
    } catch (const std::bad_alloc&) {
        return GPUHASH_ENOMEM;
    } catch (...) {
        return GPUHASH_EHIP;
    }
}

static int open_impl(const int* devices, int ndevices, gpuhash_ctx** out) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return GPUHASH_ENODEV;
    std::vector<int> ords;
    if (ndevices == 0) {
        for (int i = 0; i < count; i++) ords.push_back(i);
    } else {
        // A device may be listed more than once: each entry gets its own stream and
        // buffers and takes its own shard (rehearses the multi-device path on one GPU).
        for (int i = 0; i < ndevices; i++) {
            if (devices[i] < 0 || devices[i] >= count) return GPUHASH_EINVAL;
            ords.push_back(devices[i]);
        }
    }
    for (int o : ords) {  // the code object is gfx950-only
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, o) != hipSuccess) return GPUHASH_ENODEV;
        if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0) return GPUHASH_ENODEV;
    }
    auto* raw = new (std::nothrow) gpuhash_ctx();
    if (!raw) return GPUHASH_ENOMEM;
    // frees whatever was set up if a device fails to initialise or an allocation throws
    std::unique_ptr<gpuhash_ctx, void (*)(gpuhash_ctx*)> ctx(raw, [](gpuhash_ctx* c) {
        for (auto& d : c->devs) dev_free(d);
        delete c;
    });
    ctx->devs.resize(ords.size());
    for (size_t i = 0; i < ords.size(); i++) {
        int rc = dev_init(ctx->devs[i], ords[i], (int)i);
        if (rc) return rc;
    }
    *out = ctx.release();
    return GPUHASH_OK;
}

int gpuhash_ndevices(const gpuhash_ctx* ctx) { return ctx ? (int)ctx->devs.size() : 0; }

int gpuhash_device_count(void) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count < 0) return 0;
    return count;
}

static bool valid_policy(int policy) {
    const int base = policy & 15, flags = policy & ~15;
    return base >= GPUHASH_LAYOUT_AUTO && base <= GPUHASH_LAYOUT_LANETABLE &&
           !(flags & ~(GPUHASH_LAYOUT_TAIL_ALWAYS | GPUHASH_LAYOUT_TAIL_NEVER)) &&
           flags != (GPUHASH_LAYOUT_TAIL_ALWAYS | GPUHASH_LAYOUT_TAIL_NEVER);
}

int gpuhash_shard_range(size_t msg_len, uint64_t lower, uint64_t upper, int nshards,
                        uint64_t* out_lower, uint64_t* out_upper) {
    return gpuhash_shard_range_policy(msg_len, lower, upper, nshards, GPUHASH_LAYOUT_AUTO, out_lower, out_upper);
}

int gpuhash_shard_range_policy(size_t msg_len, uint64_t lower, uint64_t upper, int nshards, int policy,
                               uint64_t* out_lower, uint64_t* out_upper) {
    if (nshards < 1 || !out_lower || !out_upper || lower > upper || !valid_policy(policy)) return GPUHASH_EINVAL;
    if (msg_len > GPUHASH_MAX_MSG) return GPUHASH_ETOOLONG;
    try {
        // the same cost model and cut points as gpuhash_min's in-process shards under the
        // same layout policy (the cuts depend on it)
        const std::vector<Shard> sh = shard_range(msg_len, lower, upper, nshards, policy);
        int used = 0;
        for (int k = 0; k < nshards; k++) {
            const Shard& s = sh[(size_t)k];
            out_lower[k] = s.empty ? 1 : s.lo;
            out_upper[k] = s.empty ? 0 : s.hi;
            used += s.empty ? 0 : 1;
        }
        return used;
    } catch (const std::bad_alloc&) {
        return GPUHASH_ENOMEM;
    } catch (...) {
        return GPUHASH_EHIP;
    }
}

int gpuhash_set_layout_policy(gpuhash_ctx* ctx, int policy) {
    if (!ctx || !valid_policy(policy)) return GPUHASH_EINVAL;
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->policy = policy;
    return GPUHASH_OK;
}

// One slice of a search: sharded over the context's devices, each shard on its own
// host thread + stream, 16-byte host argmin.  Accumulates into st / ctx->recs.
static int run_slice(gpuhash_ctx* ctx, const uint8_t* msg, size_t msg_len, uint64_t lower,
                     uint64_t upper, uint32_t rchunk, uint64_t& bh, uint64_t& bn, bool& any,
                     gpuhash_stats& st) {
    const int n = (int)ctx->devs.size();
    std::vector<Shard> sh = shard_range(msg_len, lower, upper, n, ctx->policy);
    for (auto& d : ctx->devs) { d.used = false; d.rc = GPUHASH_OK; d.kernel_ms = 0; d.launches = 0; }
    if (n == 1) {
        ctx->devs[0].rc = dev_run(ctx->devs[0], msg, msg_len, lower, upper, rchunk, 0, nullptr, ctx->policy);
    } else {
        std::vector<std::thread> th;
        th.reserve((size_t)n);
        // Thread creation can fail (std::system_error): the shards already started are
        // joined before the error is returned, so no joinable std::thread is destroyed.
        int spawn_rc = GPUHASH_OK;
        for (int i = 0; i < n && spawn_rc == GPUHASH_OK; i++) {
            if (sh[(size_t)i].empty) continue;
            try {
            th.emplace_back([&, i] {
                Dev& d = ctx->devs[(size_t)i];
                try {
                    d.rc = dev_run(d, msg, msg_len, sh[(size_t)i].lo, sh[(size_t)i].hi, rchunk, 0, nullptr,
                                   ctx->policy);
                } catch (const std::bad_alloc&) {
                    d.used = true;
                    d.rc = GPUHASH_ENOMEM;
                } catch (...) {  // nothing may escape a std::thread (std::terminate)
                    d.used = true;
                    d.rc = GPUHASH_EHIP;
                }
            });
            } catch (const std::bad_alloc&) {
                spawn_rc = GPUHASH_ENOMEM;
            } catch (...) {
                spawn_rc = GPUHASH_EHIP;
            }
        }
        for (auto& t : th) t.join();
        if (spawn_rc) return spawn_rc;
    }
    for (auto& d : ctx->devs) {
        if (!d.used) continue;
        if (d.rc) return d.rc;
        // host argmin over the per-device 16-byte results
        if (!any || d.best_h < bh || (d.best_h == bh && d.best_n < bn)) { bh = d.best_h; bn = d.best_n; }
        any = true;
        ctx->recs.insert(ctx->recs.end(), d.recs.begin(), d.recs.end());
        st.launches += d.launches;
        st.kernel_ms += d.kernel_ms;
    }
    return GPUHASH_OK;
}

int gpuhash_min_ex(gpuhash_ctx* ctx, const uint8_t* msg, size_t msg_len, uint64_t lower,
                   uint64_t upper, uint32_t rchunk, uint64_t* out_hash, uint64_t* out_nonce) {
    if (!ctx || !out_hash || !out_nonce || (msg_len && !msg)) return GPUHASH_EINVAL;
    if (lower > upper) return GPUHASH_EINVAL;
    if (msg_len > GPUHASH_MAX_MSG) return GPUHASH_ETOOLONG;
    std::lock_guard<std::mutex> lock(ctx->mu);
    try {
        auto t0 = std::chrono::steady_clock::now();
        const uint64_t n = ctx->devs.size();
        // Searches longer than kSlicePerDevice nonces per device run as consecutive
        // slices: every launch descriptor covers <= 10^10-10^12 nonces (plan.h), so one
        // slice's plan stays a few hundred descriptors, whatever the span (a 2^64 range
        // would otherwise plan ~10^9 of them).  A slice is ~8 s of GPU work, so the
        // per-slice sync and 16-byte merge cost nothing measurable.
        // GPUHASH_SLICE_NONCES overrides the per-device slice (tests use it to exercise
        // the slice loop, including its end at 2^64-1, on oracle-sized ranges).
        uint64_t per_dev = kSlicePerDevice;
        if (const char* e = std::getenv("GPUHASH_SLICE_NONCES")) {
            const unsigned long long v = std::strtoull(e, nullptr, 10);
            if (v > 0) per_dev = v;
        }
        const uint64_t slice = per_dev > ~0ull / n ? ~0ull : per_dev * n;
        uint64_t bh = ~0ull, bn = ~0ull;
        bool any = false;
        gpuhash_stats st{};
        ctx->recs.clear();
        uint32_t ndev_used = 0;
        for (uint64_t lo = lower;;) {
            const uint64_t hi = upper - lo < slice ? upper : lo + (slice - 1);
            int rc = run_slice(ctx, msg, msg_len, lo, hi, rchunk, bh, bn, any, st);
            if (rc) return rc;
            double slice_max = 0;
            uint32_t used = 0;
            for (auto& d : ctx->devs) {
                if (!d.used) continue;
                slice_max = std::max(slice_max, d.kernel_ms);
                used++;
            }
            st.max_dev_kernel_ms += slice_max;  // devices run a slice concurrently
            ndev_used = std::max(ndev_used, used);
            if (hi == upper) break;
            lo = hi + 1;
        }
        st.ndevices = ndev_used;
        uint64_t span = upper - lower;
        st.nonces = span == ~0ull ? ~0ull : span + 1;
        st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        ctx->last = st;
        *out_hash = bh;
        *out_nonce = bn;
        return GPUHASH_OK;
    } catch (const std::bad_alloc&) {
        return GPUHASH_ENOMEM;
    } catch (...) {  // no C++ exception crosses the C ABI into a Go or Python host
        return GPUHASH_EHIP;
    }
}

int gpuhash_min(gpuhash_ctx* ctx, const uint8_t* msg, size_t msg_len, uint64_t lower,
                uint64_t upper, uint64_t* out_hash, uint64_t* out_nonce) {
    return gpuhash_min_ex(ctx, msg, msg_len, lower, upper, 0, out_hash, out_nonce);
}

int gpuhash_hash_range(gpuhash_ctx* ctx, const uint8_t* msg, size_t msg_len, uint64_t lower,
                       uint64_t count, uint64_t* out) {
    if (!ctx || !out || (msg_len && !msg) || ctx->devs.empty()) return GPUHASH_EINVAL;
    if (count == 0) return GPUHASH_OK;
    if (count > (1ull << 26) || lower + (count - 1) < lower) return GPUHASH_EINVAL;
    if (msg_len > GPUHASH_MAX_MSG) return GPUHASH_ETOOLONG;
    std::lock_guard<std::mutex> lock(ctx->mu);
    auto t0 = std::chrono::steady_clock::now();
    Dev& d = ctx->devs[0];
    for (auto& x : ctx->devs) x.used = false;
    DeviceGuard guard;
    HIPCHK(hipSetDevice(d.ord));
    unsigned long long* dd = nullptr;
    if (hipMalloc(&dd, count * sizeof(uint64_t)) != hipSuccess) return GPUHASH_ENOMEM;
    int rc;
    try {
        rc = dev_run(d, msg, msg_len, lower, lower + count - 1, 0, 1, dd, ctx->policy);
    } catch (const std::bad_alloc&) {
        rc = GPUHASH_ENOMEM;
    } catch (...) {
        rc = GPUHASH_EHIP;
    }
    if (!rc && hipMemcpy(out, dd, count * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
        rc = GPUHASH_EHIP;
    hipFree(dd);
    if (rc) return rc;
    gpuhash_stats st{};
    st.nonces = count;
    st.launches = d.launches;
    st.ndevices = 1;
    st.kernel_ms = st.max_dev_kernel_ms = d.kernel_ms;
    ctx->recs = d.recs;
    st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    ctx->last = st;
    return GPUHASH_OK;
}

uint64_t gpuhash_hash_cpu(const uint8_t* msg, size_t msg_len, uint64_t nonce) {
    return hash_host(msg, msg_len, nonce);
}

int gpuhash_last_stats(const gpuhash_ctx* ctx, gpuhash_stats* out) {
    if (!ctx || !out) return GPUHASH_EINVAL;
    std::lock_guard<std::mutex> lock(const_cast<gpuhash_ctx*>(ctx)->mu);
    *out = ctx->last;
    return GPUHASH_OK;
}

int gpuhash_last_launches(const gpuhash_ctx* ctx, gpuhash_launch_record* out, int cap) {
    if (!ctx || cap < 0 || (cap > 0 && !out)) return GPUHASH_EINVAL;
    std::lock_guard<std::mutex> lock(const_cast<gpuhash_ctx*>(ctx)->mu);
    const int n = (int)ctx->recs.size();
    for (int i = 0; i < n && i < cap; i++) out[i] = ctx->recs[(size_t)i];
    return n;
}

void gpuhash_close(gpuhash_ctx* ctx) {
    if (!ctx) return;
    for (auto& d : ctx->devs) dev_free(d);
    delete ctx;
}

const char* gpuhash_strerror(int rc) {
    switch (rc) {
        case GPUHASH_OK: return "ok";
        case GPUHASH_EINVAL: return "invalid argument (null pointer, lower > upper, or bad device list)";
        case GPUHASH_ENODEV: return "no usable gfx950 (MI355X) device";
        case GPUHASH_EHIP: return "HIP runtime error or kernel launch failure";
        case GPUHASH_ETOOLONG: return "message longer than GPUHASH_MAX_MSG";
        case GPUHASH_ENOMEM: return "out of device or host memory";
        default: return "unknown gpuhash error";
    }
}

#ifndef GPUHASH_BUILD_ID
#define GPUHASH_BUILD_ID "unknown"
#endif

const char* gpuhash_version(void) {
#ifdef GPUHASH_TIE_TEST_BITS
    return "gpuhash 0.3 gfx950 build=" GPUHASH_BUILD_ID " TIE-TEST (truncated keys; test build only)";
#else
    return "gpuhash 0.3 gfx950 build=" GPUHASH_BUILD_ID;
#endif
}

}  // extern "C"
