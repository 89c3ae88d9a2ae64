// engine.hip -- the C-ABI (include/fqengine.h) over the gfx950 kernels.
//
// No CPU fallback: creation fails with FQ_E_NO_DEVICE unless a gfx950 device is present.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <deque>
#include <mutex>
#include <unordered_map>
#include <sys/mman.h>
#include <string>

// profiling only (FQ_PROF_NO_EGRESS=1): raw packs copy no output text back and report none, to
// time the pipeline without its device-to-host leg (the outputs are empty)
static bool prof_no_egress() {
    static const bool on = std::getenv("FQ_PROF_NO_EGRESS") != nullptr;
    return on;
}

#include "engine_internal.h"

// Tile list the fast kernel hands to the general kernel (one per concurrently running launch).
struct Scratch {
    int* slow_tiles = nullptr;
    int* slow_count = nullptr;
    size_t slow_cap = 0;
};

// One in-flight pack of the asynchronous pipeline (fq_engine_submit / fq_engine_poll): its own
// device copy of the batch, result records and hand-off list, and the events that order
//   H2D (stream in) -> kernels (compute stream) -> D2H of the records (stream out).
struct Slot {
    uint8_t* d_rows = nullptr;  // 4 planes of fq_batch_bytes(max_batch, max_stride)
    uint16_t* d_lens = nullptr;  // 2 x max_batch
    uint8_t* d_flags = nullptr;  // max_batch per-pair FQ_BF_* flags
    fq_read_result* d_res = nullptr;
    Scratch scratch;
    hipEvent_t ev_in = nullptr, ev_kern = nullptr, ev_done = nullptr;
    // FASTQ-text packs (fq_engine_submit_text): per mate text, records, output text, sizes, offsets
    char* d_text[2] = {nullptr, nullptr};
    char* d_out[2] = {nullptr, nullptr};
    size_t text_cap[2] = {0, 0};
    fq_text_rec* d_trec[2] = {nullptr, nullptr};
    uint32_t* d_tsize[2] = {nullptr, nullptr};
    uint32_t* d_toff[2] = {nullptr, nullptr};
    size_t trec_cap = 0;
    void* d_scan = nullptr;
    size_t scan_bytes = 0;
    unsigned long long* d_total = nullptr;  // [2]
    unsigned long long* h_total = nullptr;  // pinned [2]
    fq_text_out* text_out = nullptr;        // the pending text pack's output descriptor
    // raw windows (fq_engine_raw_*): line index, block counts / bases, indexing state, adapter entries
    uint32_t* d_lines[2] = {nullptr, nullptr};
    uint32_t* d_bcnt[2] = {nullptr, nullptr};
    uint32_t* d_bbase[2] = {nullptr, nullptr};
    fq_raw_state* d_rstate = nullptr;  // [2]
    fq_raw_state* h_rstate = nullptr;  // pinned [2]
    char* d_ad[2] = {nullptr, nullptr};
    size_t ad_cap = 0;
    bool raw_ready = false;
    hipEvent_t ev_idx = nullptr;
    fq_raw_out* raw_out = nullptr;  // the pending raw pack's output descriptor
    uint64_t raw_n[2] = {0, 0};     // the window's raw bytes
    int* d_err = nullptr;  // this pack's device error word (cleared at submit, set by its kernels)
    int* h_err = nullptr;  // pinned: d_err as of this pack's kernels
    bool busy = false;      // events recorded and not yet waited for
    // raw packs: the output text is copied back once its size is known (issue_copies)
    bool copy_pending = false;
    char* copy_dst[2] = {nullptr, nullptr};
    size_t copy_cap[2] = {0, 0};
};

// A submitted pack, in submission order, until fq_engine_poll reports it.
struct Pending {
    uint64_t seq_no;
    int slot;
    bool done;  // its slot's events completed (the slot may already serve a later pack)
    int err;
};

static const int kSlots = 3;     // host packs: H2D(k+1) || kernels(k) || D2H(k-1)
static const int kRawSlots = 8;  // raw windows: up to 3 enqueued + 5 launched, copies queued each way

struct fq_engine {
    fq_params p;
    int device = 0;
    int cus = 0;
    char arch[64] = {0};
    int32_t max_batch = 0, max_stride = 0;
    hipStream_t stream = nullptr;
    unsigned long long* acc = nullptr;      // accumulator in use
    unsigned long long* own_acc = nullptr;  // the engine's own buffer
    unsigned long long* xfix = nullptr;     // the fast kernels' exotic-byte Stats moves (fq_xfix_words)
    size_t acc_words = 0;
    int* err = nullptr;
    // host-memory path: pipeline slots and their streams
    Slot slots[kRawSlots];  // (host packs use the first kSlots)
    std::deque<Pending> pending;
    hipStream_t s_in = nullptr, s_out = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool fast = false;  // pe_fast kernel usable for these params
    Scratch scratch;    // hand-off list of fq_engine_process_device
    bool timed = false;
    // raw stream (fq_engine_raw_*): window / carry capacity, index stream, windows not yet launched
    bool raw = false;
    uint64_t raw_wcap = 0, raw_ccap = 0;
    uint32_t raw_nblocks = 0;
    hipStream_t s_idx = nullptr;
    std::deque<int> raw_queued;
    int raw_prev_slot = -1;
    fq_dup* dup = nullptr;    // duplication table fed by every pack (-d)
    uint64_t calls = 0;       // order of process / process_device packs for the table
    std::string last_error;
};

static std::string g_create_error;

// FQ_ENGINE_TIMING=1: creation steps and the raw stream's one-time set-up on stderr (profiling)
static bool engine_timing() {
    static const bool on = std::getenv("FQ_ENGINE_TIMING") != nullptr;
    return on;
}
static double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

// Raw-window copies of the engines that share one GPU (and so one PCIe link) run one after another
// in call order: each engine's host-to-device copies wait for the last one another engine enqueued
// on the device (and likewise its device-to-host copies).  Left to share the link, the copies of a
// window that is due would finish only with those of the windows enqueued behind it on the other
// engines (the raw stream launches windows in order), so several engines on one GPU ran slower than
// one.  Engines on different GPUs never wait for each other.
struct LinkChain {
    std::mutex m;
    hipEvent_t in = nullptr, out = nullptr;  // the last copies enqueued on the device
    const fq_engine *in_owner = nullptr, *out_owner = nullptr;
};
static LinkChain& link_chain(int device) {
    static LinkChain chains[64];
    return chains[device & 63];
}

static int fail(fq_engine* e, int code, const std::string& msg) {
    if (e) e->last_error = msg;
    else g_create_error = msg;
    return code;
}

static int hip_fail(fq_engine* e, hipError_t err, const char* what) {
    return fail(e, FQ_E_HIP, std::string(what) + ": " + hipGetErrorString(err));
}

#define HIP_TRY(e, call)                                       \
    do {                                                       \
        hipError_t _err = (call);                              \
        if (_err != hipSuccess) return hip_fail(e, _err, #call); \
    } while (0)

static int validate_params(const fq_params* p, std::string& why) {
    if (p->max_cycles < 1 || p->max_cycles > FQ_MAX_CYCLES_LIMIT) return why = "max_cycles must be in [1, 4096]", FQ_E_INVALID;
    if (p->insert_size_max < 0 || p->insert_size_max > 100000) return why = "bad insert_size_max", FQ_E_INVALID;
    if (p->cut_front && p->cut_front_window < 1) return why = "cut_front window must be >= 1", FQ_E_INVALID;
    if (p->cut_right && p->cut_right_window < 1) return why = "cut_right window must be >= 1", FQ_E_INVALID;
    if (p->cut_tail && p->cut_tail_window < 1) return why = "cut_tail window must be >= 1", FQ_E_INVALID;
    if (p->polyg_enabled && p->polyg_one_mismatch_per < 1) return why = "polyG one-mismatch-per must be >= 1", FQ_E_INVALID;
    if (p->polyx_enabled && p->polyx_one_mismatch_per < 1) return why = "polyX one-mismatch-per must be >= 1", FQ_E_INVALID;
    if (p->adapter1_len < 0 || p->adapter1_len > FQ_MAX_ADAPTER || p->adapter2_len < 0 ||
        p->adapter2_len > FQ_MAX_ADAPTER)
        return why = "bad adapter length", FQ_E_INVALID;
    return FQ_OK;
}

static int ensure_scratch(fq_engine* e, Scratch& sc, size_t ntiles, bool sync_device) {
    if (!sc.slow_count) HIP_TRY(e, hipMalloc(&sc.slow_count, sizeof(int)));
    if (ntiles <= sc.slow_cap) return FQ_OK;
    // the old list may still be read by a launch in flight
    if (sync_device) HIP_TRY(e, hipDeviceSynchronize());
    if (sc.slow_tiles) HIP_TRY(e, hipFree(sc.slow_tiles));
    sc.slow_tiles = nullptr;
    sc.slow_cap = 0;
    HIP_TRY(e, hipMalloc(&sc.slow_tiles, ntiles * sizeof(int)));
    sc.slow_cap = ntiles;
    return FQ_OK;
}

static void free_scratch(Scratch& sc) {
    if (sc.slow_tiles) (void)hipFree(sc.slow_tiles);
    if (sc.slow_count) (void)hipFree(sc.slow_count);
    sc = Scratch();
}

static void free_slot(Slot& s) {
    if (s.d_rows) (void)hipFree(s.d_rows);
    if (s.d_lens) (void)hipFree(s.d_lens);
    if (s.d_flags) (void)hipFree(s.d_flags);
    if (s.d_res) (void)hipFree(s.d_res);
    for (int m = 0; m < 2; ++m) {
        if (s.d_text[m]) (void)hipFree(s.d_text[m]);
        if (s.d_out[m]) (void)hipFree(s.d_out[m]);
        if (s.d_trec[m]) (void)hipFree(s.d_trec[m]);
        if (s.d_tsize[m]) (void)hipFree(s.d_tsize[m]);
        if (s.d_toff[m]) (void)hipFree(s.d_toff[m]);
    }
    if (s.d_scan) (void)hipFree(s.d_scan);
    if (s.d_total) (void)hipFree(s.d_total);
    if (s.h_total) (void)hipHostFree(s.h_total);
    for (int m = 0; m < 2; ++m) {
        if (s.d_lines[m]) (void)hipFree(s.d_lines[m]);
        if (s.d_bcnt[m]) (void)hipFree(s.d_bcnt[m]);
        if (s.d_bbase[m]) (void)hipFree(s.d_bbase[m]);
        if (s.d_ad[m]) (void)hipFree(s.d_ad[m]);
    }
    if (s.d_rstate) (void)hipFree(s.d_rstate);
    if (s.h_rstate) (void)hipHostFree(s.h_rstate);
    if (s.ev_idx) (void)hipEventDestroy(s.ev_idx);
    if (s.d_err) (void)hipFree(s.d_err);
    if (s.h_err) (void)hipHostFree(s.h_err);
    if (s.ev_in) (void)hipEventDestroy(s.ev_in);
    if (s.ev_kern) (void)hipEventDestroy(s.ev_kern);
    if (s.ev_done) (void)hipEventDestroy(s.ev_done);
    free_scratch(s.scratch);
    s = Slot();
}

static int alloc_slot(fq_engine* e, Slot& s) {
    if (s.d_rows) return FQ_OK;
    const size_t rows = (size_t)4 * fq_batch_bytes(e->max_batch, e->max_stride);
    HIP_TRY(e, hipMalloc(&s.d_rows, rows));
    HIP_TRY(e, hipMalloc(&s.d_lens, (size_t)2 * e->max_batch * sizeof(uint16_t)));
    HIP_TRY(e, hipMalloc(&s.d_flags, (size_t)e->max_batch + 1));
    HIP_TRY(e, hipMalloc(&s.d_res, (size_t)2 * e->max_batch * sizeof(fq_read_result)));
    HIP_TRY(e, hipMalloc(&s.d_err, sizeof(int)));
    HIP_TRY(e, hipHostMalloc((void**)&s.h_err, sizeof(int), hipHostMallocDefault));
    *s.h_err = 0;
    HIP_TRY(e, hipEventCreateWithFlags(&s.ev_in, hipEventDisableTiming));
    HIP_TRY(e, hipEventCreateWithFlags(&s.ev_kern, hipEventDisableTiming));
    HIP_TRY(e, hipEventCreateWithFlags(&s.ev_done, hipEventDisableTiming));
    return FQ_OK;
}

extern "C" {

int fq_engine_create(const fq_params* params, int device, int32_t max_batch, int32_t max_stride, fq_engine** out) {
    if (!params || !out || max_batch < 0 || max_stride < 0 || (max_stride & 15))
        return fail(nullptr, FQ_E_INVALID, "fq_engine_create: bad arguments (stride must be a multiple of 16)");
    *out = nullptr;
    std::string why;
    if (validate_params(params, why) != FQ_OK) return fail(nullptr, FQ_E_INVALID, why);
    // FQ_ENGINE_TIMING=1: the creation's steps on stderr (profiling: start-up of the tool)
    const bool timing = engine_timing();
    const auto t0 = std::chrono::steady_clock::now();
    auto stamp = [&](const char* what) {
        if (timing)
            std::fprintf(stderr, "fq_engine_create: %s at %.4f s\n", what,
                         std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    };
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(nullptr, FQ_E_NO_DEVICE, "no HIP device visible (the engine has no CPU fallback)");
    if (device < 0 || device >= ndev) return fail(nullptr, FQ_E_NO_DEVICE, "device id out of range");
    stamp("runtime up (hipGetDeviceCount)");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess)
        return fail(nullptr, FQ_E_NO_DEVICE, "hipGetDeviceProperties failed");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(nullptr, FQ_E_NO_DEVICE, std::string("device is ") + prop.gcnArchName + ", engine is built for gfx950");
    fq_engine* e = new fq_engine();
    e->p = *params;
    e->device = device;
    e->cus = prop.multiProcessorCount;
    std::snprintf(e->arch, sizeof e->arch, "%s", prop.gcnArchName);
    e->max_batch = max_batch;
    e->max_stride = max_stride;
    e->acc_words = fq_acc_words(params->insert_size_max, params->max_cycles);
    auto bail = [&](int rc) {
        g_create_error = e->last_error;
        fq_engine_destroy(e);
        return rc;
    };
    hipError_t he;
    if ((he = hipSetDevice(device)) != hipSuccess) return bail(hip_fail(e, he, "hipSetDevice"));
    for (hipStream_t* s : {&e->stream, &e->s_in, &e->s_out})
        if ((he = hipStreamCreateWithFlags(s, hipStreamNonBlocking)) != hipSuccess)
            return bail(hip_fail(e, he, "hipStreamCreate"));
    if ((he = hipMalloc(&e->own_acc, e->acc_words * 8)) != hipSuccess) return bail(hip_fail(e, he, "hipMalloc acc"));
    e->acc = e->own_acc;
    if ((he = hipMalloc(&e->err, sizeof(int))) != hipSuccess) return bail(hip_fail(e, he, "hipMalloc err"));
    if ((he = hipMemset(e->acc, 0, e->acc_words * 8)) != hipSuccess) return bail(hip_fail(e, he, "hipMemset"));
    const size_t xw = fq_xfix_words(params->max_cycles);
    if ((he = hipMalloc(&e->xfix, xw * 8)) != hipSuccess) return bail(hip_fail(e, he, "hipMalloc xfix"));
    if ((he = hipMemset(e->xfix, 0, xw * 8)) != hipSuccess) return bail(hip_fail(e, he, "hipMemset"));
    if ((he = hipMemset(e->err, 0, sizeof(int))) != hipSuccess) return bail(hip_fail(e, he, "hipMemset"));
    stamp("streams and accumulators");
    // the first pipeline slot up front, so an engine that cannot hold one pack fails here
    if (max_batch > 0 && max_stride > 0 && alloc_slot(e, e->slots[0]) != FQ_OK) return bail(FQ_E_HIP);
    stamp("first slot");
    if ((he = hipEventCreate(&e->ev0)) != hipSuccess) return bail(hip_fail(e, he, "hipEventCreate"));
    if ((he = hipEventCreate(&e->ev1)) != hipSuccess) return bail(hip_fail(e, he, "hipEventCreate"));
    if (fq_pack_kernel_lds_bytes(e->p) > 160 * 1024)
        return bail(fail(e, FQ_E_INVALID, "insert_size_max too large for the LDS-privatised accumulators"));
    if ((he = fq_pack_kernel_set_lds(e->p)) != hipSuccess) return bail(hip_fail(e, he, "hipFuncSetAttribute"));
    const char* force_general = std::getenv("FQ_ENGINE_GENERAL_ONLY");
    e->fast = fq_pe_fast_supported(e->p) && !(force_general && force_general[0] == '1');
    stamp("general kernel attributes");
    if (e->fast) {
        if ((he = fq_pe_fast_prepare()) != hipSuccess) return bail(hip_fail(e, he, "hipFuncSetAttribute fast"));
    }
    stamp("fast kernel attributes");
    *out = e;
    return FQ_OK;
}

int fq_engine_destroy(fq_engine* e) {
    if (!e) return FQ_OK;
    (void)hipSetDevice(e->device);
    (void)hipDeviceSynchronize();
    {
        LinkChain& lc = link_chain(e->device);  // (its events are about to go)
        std::lock_guard<std::mutex> g(lc.m);
        if (lc.in_owner == e) lc.in = nullptr, lc.in_owner = nullptr;
        if (lc.out_owner == e) lc.out = nullptr, lc.out_owner = nullptr;
    }
    if (e->own_acc) (void)hipFree(e->own_acc);
    if (e->xfix) (void)hipFree(e->xfix);
    if (e->err) (void)hipFree(e->err);
    for (Slot& s : e->slots) free_slot(s);
    free_scratch(e->scratch);
    if (e->ev0) (void)hipEventDestroy(e->ev0);
    if (e->ev1) (void)hipEventDestroy(e->ev1);
    for (hipStream_t s : {e->stream, e->s_in, e->s_out, e->s_idx})
        if (s) (void)hipStreamDestroy(s);
    delete e;
    return FQ_OK;
}

static int grid_for(const fq_engine* e, int n) {
    const size_t lds = fq_pack_kernel_lds_bytes(e->p);
    int per_cu = (int)((160 * 1024) / (lds ? lds : 1));
    if (per_cu < 1) per_cu = 1;
    if (per_cu > 8) per_cu = 8;
    const int cap = e->cus * per_cu;
    const int need = (n + kPackThreads - 1) / kPackThreads;
    return need < cap ? (need > 0 ? need : 1) : cap;
}

// Enqueues the kernels of one batch on stream s.  `sc` is the hand-off list of this launch; it
// must not be shared with a launch that can run concurrently (different stream).
static int launch(fq_engine* e, const fq_batch& db, fq_read_result* dres, hipStream_t s, Scratch& sc, bool timed,
                  bool sync_device_on_grow, uint64_t order, int* derr) {
    if (db.n <= 0) return FQ_OK;
    if (e->dup) {  // Duplicate::statPair / statRead run on the untrimmed reads (src/peprocessor.cpp:279-281)
        const int rc = fq_dup_pack(e->dup, db, e->p.paired, order, s);
        if (rc != FQ_OK) return fail(e, rc, std::string("duplication analysis: ") + fq_dup_error(e->dup));
    }
    // (index-filtered pairs are handed to the general kernel one by one)
    if (e->fast) {
        // hand-off list: pair / read indices, reserved a tile's worth (<= 64) at a time, at most
        // one reservation per tile, so at most n + 64 slots (holes included)
        const size_t nitems = (size_t)db.n + 64 + 1;
        int rc = ensure_scratch(e, sc, nitems, sync_device_on_grow);
        if (rc != FQ_OK) return rc;
        HIP_TRY(e, hipMemsetAsync(sc.slow_count, 0, sizeof(int), s));
        if (timed) HIP_TRY(e, hipEventRecord(e->ev0, s));
        HIP_TRY(e, fq_launch_pe_fast(e->p, db, dres, e->acc, sc.slow_tiles, sc.slow_count, e->xfix, e->cus, s));
        HIP_TRY(e, fq_launch_xfix_fold(e->acc + fq_acc_stats_offset(e->p.insert_size_max, e->p.max_cycles, 0), e->xfix,
                                       e->p.max_cycles, s));
        // (the hand-off list's length is known on the device only: as many workgroups as the
        // batch could need, at the occupancy the kernel's LDS allows; empty ones exit at once)
        HIP_TRY(e, fq_launch_pack_kernel(e->p, db, dres, e->acc, derr, grid_for(e, db.n), s, sc.slow_tiles,
                                         sc.slow_count));
    } else {
        if (timed) HIP_TRY(e, hipEventRecord(e->ev0, s));
        HIP_TRY(e, fq_launch_pack_kernel(e->p, db, dres, e->acc, derr, grid_for(e, db.n), s));
    }
    if (timed) {
        HIP_TRY(e, hipEventRecord(e->ev1, s));
        e->timed = true;
    }
    return FQ_OK;
}

static int check_err(fq_engine* e) {
    int h = 0;
    HIP_TRY(e, hipMemcpy(&h, e->err, sizeof(int), hipMemcpyDeviceToHost));
    if (h) {
        HIP_TRY(e, hipMemset(e->err, 0, sizeof(int)));
        return fail(e, FQ_E_TOO_LONG, "a read is longer than max_cycles or the row stride");
    }
    return FQ_OK;
}

// Raw packs' copies back, exactly sized: a pack's kernels end by copying its output sizes to the
// host (on the compute stream, event ev_kern); once they are in, its text + adapter entries are
// copied back on the out stream (in submission order; the link chain orders the copies of engines
// sharing a GPU).  Copying the capacity bound instead carried the gap left by trimmed and dropped
// records and, with -m, mate 1's whole input-sized bound for its few entry bytes (the e2e C4 leg's
// copies back took 1.44x the C3 leg's).  upto = a slot: waits for the sizes of the packs up to
// and including that slot's; -1: issues what is ready, stopping at the first pack whose sizes are
// not in; -2: waits for all.
static int issue_copies(fq_engine* e, int upto) {
    for (Pending& q : e->pending) {
        if (q.done) continue;
        Slot& s = e->slots[q.slot];
        if (s.copy_pending) {
            if (upto == -1) {
                const hipError_t st = hipEventQuery(s.ev_kern);
                if (st == hipErrorNotReady) break;
                if (st != hipSuccess) return hip_fail(e, st, "hipEventQuery");
            } else {
                HIP_TRY(e, hipEventSynchronize(s.ev_kern));
            }
            s.copy_pending = false;
            LinkChain& lc = link_chain(e->device);
            std::lock_guard<std::mutex> g(lc.m);
            if (lc.out && lc.out_owner != e) HIP_TRY(e, hipStreamWaitEvent(e->s_out, lc.out, 0));
            for (int m = 0; m < 2 && !prof_no_egress(); ++m) {
                if (!s.copy_dst[m]) continue;
                const unsigned long long ad = s.h_total[2 + m];  // (~0: the entries overflowed, reported at retire)
                const size_t bytes = std::min<size_t>(s.copy_cap[m], (size_t)s.h_total[m] + (ad == ~0ull ? 0 : (size_t)ad));
                if (bytes) HIP_TRY(e, hipMemcpyAsync(s.copy_dst[m], s.d_out[m], bytes, hipMemcpyDeviceToHost, e->s_out));
            }
            HIP_TRY(e, hipEventRecord(s.ev_done, e->s_out));
            lc.out = s.ev_done, lc.out_owner = e;
        }
        if (q.slot == upto) break;
    }
    return FQ_OK;
}

// Waits for slot k's pack (if any) and records its completion in the pending list.
static int retire_slot(fq_engine* e, int k) {
    Slot& s = e->slots[k];
    if (!s.busy) return FQ_OK;
    if (s.copy_pending) {
        const int rc = issue_copies(e, k);
        if (rc != FQ_OK) return rc;
    }
    HIP_TRY(e, hipEventSynchronize(s.ev_done));
    s.busy = false;
    for (Pending& q : e->pending)
        if (q.slot == k && !q.done) {
            q.done = true;
            q.err = *s.h_err;
        }
    if (s.text_out) {  // a text pack: its output sizes are in now
        s.text_out->bytes[0] = s.h_total[0];
        s.text_out->bytes[1] = s.h_total[1];
        s.text_out = nullptr;
    }
    if (s.raw_out) {  // a raw pack: its trimmed-adapter entries follow the output text
        fq_raw_out* o = s.raw_out;
        s.raw_out = nullptr;
        for (int m = 0; m < 2; ++m) {
            o->adapter_bytes[m] = s.h_total[2 + m];
            if (o->adapter_bytes[m] == ~0ull) return fail(e, FQ_E_INVALID, "raw pack: adapter entries exceed the output copy");
            if (prof_no_egress()) o->adapter_bytes[m] = o->text.bytes[m] = 0;
        }
    }
    return FQ_OK;
}

// a text pack's output is at most its input plus the final line terminator an input may lack
static const size_t kTextSlack = 16;
// -m: mate 0's output is the merged stream, at most both mates' input plus a merged name's tag
// ("_merged_<m1>_<m2>", < 24 bytes) per pair
static size_t merged_cap(uint64_t text1, uint64_t text2, size_t pairs) {
    return (size_t)text1 + (size_t)text2 + 24 * pairs + kTextSlack;
}

// the output text of a text / raw pack: out1 (+ out2), or (-m) the merged stream into mate 0's buffer
static int launch_text_out(fq_engine* e, Slot& s, int n) {
    const bool pe = e->p.paired;
    if (pe && e->p.merge_enabled) {
        HIP_TRY(e, fq_launch_merge_out(s.d_text[0], s.d_text[1], s.d_trec[0], s.d_trec[1], s.d_res, n, e->p.discard_unmerged,
                                       s.d_tsize[0], s.d_toff[0], s.d_scan, s.scan_bytes, s.d_out[0], s.d_total, e->stream));
        HIP_TRY(e, hipMemsetAsync(s.d_total + 1, 0, sizeof(unsigned long long), e->stream));
        return FQ_OK;
    }
    for (int m = 0; m < (pe ? 2 : 1); ++m)
        HIP_TRY(e, fq_launch_text_out(s.d_text[m], s.d_trec[m], s.d_res, n, pe ? 1 : 0, m, s.d_tsize[m], s.d_toff[m],
                                      s.d_scan, s.scan_bytes, s.d_out[m], s.d_total + m, e->stream));
    if (!pe) HIP_TRY(e, hipMemsetAsync(s.d_total + 1, 0, sizeof(unsigned long long), e->stream));
    return FQ_OK;
}

// device buffers of a text pack (grown on demand; growing frees the old ones, which waits for the
// device, so steady-state packs of similar size reuse them)
static int ensure_text(fq_engine* e, Slot& s, const fq_text_batch* tb) {
    const bool pe = e->p.paired;
    const bool mrg = pe && e->p.merge_enabled;
    for (int m = 0; m < (pe ? 2 : 1); ++m) {
        size_t need = tb->text_bytes[m] + kTextSlack;
        // (-m: mate 0's output buffer takes the merged stream; the sizes go together)
        if (mrg && m == 0) need = merged_cap(tb->text_bytes[0], tb->text_bytes[1], (size_t)tb->n);
        if (need > s.text_cap[m]) {
            s.raw_ready = false;  // (the raw-window buffers are re-made by ensure_raw)
            if (s.d_text[m]) (void)hipFree(s.d_text[m]);
            if (s.d_out[m]) (void)hipFree(s.d_out[m]);
            s.d_text[m] = s.d_out[m] = nullptr;
            s.text_cap[m] = 0;
            const size_t cap = need + need / 8;
            HIP_TRY(e, hipMalloc(&s.d_text[m], cap));
            HIP_TRY(e, hipMalloc(&s.d_out[m], cap));
            s.text_cap[m] = cap;
        }
    }
    if ((size_t)tb->n > s.trec_cap || !s.d_total) {
        s.raw_ready = false;
        const size_t cap = (size_t)tb->n + (size_t)tb->n / 8 + 1;
        for (int m = 0; m < 2; ++m) {
            if (s.d_trec[m]) (void)hipFree(s.d_trec[m]);
            if (s.d_tsize[m]) (void)hipFree(s.d_tsize[m]);
            if (s.d_toff[m]) (void)hipFree(s.d_toff[m]);
            s.d_trec[m] = nullptr;
            s.d_tsize[m] = s.d_toff[m] = nullptr;
        }
        if (s.d_scan) (void)hipFree(s.d_scan);
        s.d_scan = nullptr;
        s.trec_cap = 0;
        for (int m = 0; m < 2; ++m) {
            HIP_TRY(e, hipMalloc(&s.d_trec[m], cap * sizeof(fq_text_rec)));
            HIP_TRY(e, hipMalloc(&s.d_tsize[m], cap * sizeof(uint32_t)));
            HIP_TRY(e, hipMalloc(&s.d_toff[m], cap * sizeof(uint32_t)));
        }
        s.scan_bytes = fq_text_scan_temp_bytes((int)cap);
        HIP_TRY(e, hipMalloc(&s.d_scan, s.scan_bytes ? s.scan_bytes : 1));
        if (!s.d_total) HIP_TRY(e, hipMalloc(&s.d_total, 4 * sizeof(unsigned long long)));
        if (!s.h_total) HIP_TRY(e, hipHostMalloc((void**)&s.h_total, 4 * sizeof(unsigned long long), hipHostMallocDefault));
        s.trec_cap = cap;
    }
    return FQ_OK;
}

static int validate_host_batch(fq_engine* e, const fq_batch* hb) {
    const bool pe = e->p.paired;
    if (hb->n < 0 || hb->n > e->max_batch || hb->stride <= 0 || hb->stride > e->max_stride || (hb->stride & 15))
        return fail(e, FQ_E_INVALID, "batch exceeds the engine's max_batch/max_stride (or stride % 16 != 0)");
    if (!hb->seq1 || !hb->qual1 || !hb->len1 || (pe && (!hb->seq2 || !hb->qual2 || !hb->len2)))
        return fail(e, FQ_E_INVALID, "missing batch arrays");
    // -c hands the host the overlap offset of a corrected pair in a 16-bit signed record field
    if (e->p.correction_enabled && hb->stride > 32768)
        return fail(e, FQ_E_INVALID, "-c takes reads of at most 32767 bases (the record's overlap offset is 16-bit)");
    // (read lengths are checked on the device: a read longer than max_cycles or the stride sets
    // the pack's error word, which fq_engine_poll reports as FQ_E_TOO_LONG)
    return FQ_OK;
}

int fq_engine_submit(fq_engine* e, const fq_batch* hb, fq_read_result* results, uint64_t seq_no) {
    if (!e || !hb || !results) return FQ_E_INVALID;
    int rc = validate_host_batch(e, hb);
    if (rc != FQ_OK) return rc;
    if (hb->n == 0) {  // nothing to move: complete at once, in order
        e->pending.push_back(Pending{seq_no, -1, true, 0});
        return FQ_OK;
    }
    HIP_TRY(e, hipSetDevice(e->device));
    // the slot after the newest pack's (round robin), once its previous pack has drained
    int k = 0;
    for (auto it = e->pending.rbegin(); it != e->pending.rend(); ++it)
        if (it->slot >= 0) {
            k = (it->slot + 1) % kSlots;
            break;
        }
    if ((rc = retire_slot(e, k)) != FQ_OK) return rc;
    Slot& s = e->slots[k];
    if ((rc = alloc_slot(e, s)) != FQ_OK) return rc;
    const bool pe = e->p.paired;
    const size_t rowbytes = fq_batch_bytes(hb->n, hb->stride);
    const size_t plane = fq_batch_bytes(e->max_batch, e->max_stride);
    fq_batch db{};
    db.n = hb->n;
    db.stride = hb->stride;
    db.seq1 = s.d_rows;
    db.qual1 = s.d_rows + plane;
    db.len1 = s.d_lens;
    db.seq2 = pe ? s.d_rows + 2 * plane : nullptr;
    db.qual2 = pe ? s.d_rows + 3 * plane : nullptr;
    db.len2 = pe ? s.d_lens + e->max_batch : nullptr;
    // H2D on the copy-in stream (overlaps the previous pack's kernels when the host batch is pinned)
    HIP_TRY(e, hipMemcpyAsync((void*)db.seq1, hb->seq1, rowbytes, hipMemcpyHostToDevice, e->s_in));
    HIP_TRY(e, hipMemcpyAsync((void*)db.qual1, hb->qual1, rowbytes, hipMemcpyHostToDevice, e->s_in));
    HIP_TRY(e, hipMemcpyAsync((void*)db.len1, hb->len1, (size_t)hb->n * 2, hipMemcpyHostToDevice, e->s_in));
    if (pe) {
        HIP_TRY(e, hipMemcpyAsync((void*)db.seq2, hb->seq2, rowbytes, hipMemcpyHostToDevice, e->s_in));
        HIP_TRY(e, hipMemcpyAsync((void*)db.qual2, hb->qual2, rowbytes, hipMemcpyHostToDevice, e->s_in));
        HIP_TRY(e, hipMemcpyAsync((void*)db.len2, hb->len2, (size_t)hb->n * 2, hipMemcpyHostToDevice, e->s_in));
    }
    if (hb->flags) {
        db.flags = s.d_flags;
        HIP_TRY(e, hipMemcpyAsync((void*)db.flags, hb->flags, (size_t)hb->n, hipMemcpyHostToDevice, e->s_in));
    }
    HIP_TRY(e, hipEventRecord(s.ev_in, e->s_in));
    // kernels on the compute stream (one accumulator: the packs' kernels run in order)
    HIP_TRY(e, hipStreamWaitEvent(e->stream, s.ev_in, 0));
    HIP_TRY(e, hipMemsetAsync(s.d_err, 0, sizeof(int), e->stream));
    if ((rc = launch(e, db, s.d_res, e->stream, s.scratch, false, false, seq_no, s.d_err)) != FQ_OK) return rc;
    HIP_TRY(e, hipEventRecord(s.ev_kern, e->stream));
    // D2H of the records (and of the error flag) on the copy-out stream
    HIP_TRY(e, hipStreamWaitEvent(e->s_out, s.ev_kern, 0));
    const size_t nres = (size_t)hb->n * (pe ? 2 : 1);
    if (nres)
        HIP_TRY(e, hipMemcpyAsync(results, s.d_res, nres * sizeof(fq_read_result), hipMemcpyDeviceToHost, e->s_out));
    HIP_TRY(e, hipMemcpyAsync(s.h_err, s.d_err, sizeof(int), hipMemcpyDeviceToHost, e->s_out));
    HIP_TRY(e, hipEventRecord(s.ev_done, e->s_out));
    s.busy = true;
    e->pending.push_back(Pending{seq_no, k, false, 0});
    return FQ_OK;
}

int fq_engine_submit_text(fq_engine* e, const fq_text_batch* tb, fq_read_result* results, fq_text_out* out,
                          uint64_t seq_no) {
    if (!e || !tb || !results || !out) return FQ_E_INVALID;
    const bool pe = e->p.paired;
    if (tb->n < 0 || tb->n > e->max_batch || tb->stride <= 0 || tb->stride > e->max_stride || (tb->stride & 15))
        return fail(e, FQ_E_INVALID, "text pack exceeds the engine's max_batch/max_stride (or stride % 16 != 0)");
    if (e->p.correction_enabled || e->p.umi_front1 > 0 || e->p.umi_front2 > 0 ||
        (e->p.merge_enabled && e->p.discard_unmerged))
        return fail(e, FQ_E_INVALID, "text packs take no -c, UMI or --discard_unmerged options");
    for (int m = 0; m < (pe ? 2 : 1); ++m)
        if (tb->n > 0 && (!tb->text[m] || !tb->rec[m] || !out->text[m]))
            return fail(e, FQ_E_INVALID, "missing text pack arrays");
    const bool mrg = pe && e->p.merge_enabled;
    out->bytes[0] = out->bytes[1] = 0;
    if (tb->n == 0) {
        e->pending.push_back(Pending{seq_no, -1, true, 0});
        return FQ_OK;
    }
    HIP_TRY(e, hipSetDevice(e->device));
    int k = 0;
    for (auto it = e->pending.rbegin(); it != e->pending.rend(); ++it)
        if (it->slot >= 0) {
            k = (it->slot + 1) % kSlots;
            break;
        }
    int rc = retire_slot(e, k);
    if (rc != FQ_OK) return rc;
    Slot& s = e->slots[k];
    if ((rc = alloc_slot(e, s)) != FQ_OK) return rc;
    if ((rc = ensure_text(e, s, tb)) != FQ_OK) return rc;
    const size_t plane = fq_batch_bytes(e->max_batch, e->max_stride);
    fq_batch db{};
    db.n = tb->n;
    db.stride = tb->stride;
    db.seq1 = s.d_rows;
    db.qual1 = s.d_rows + plane;
    db.len1 = s.d_lens;
    db.seq2 = pe ? s.d_rows + 2 * plane : nullptr;
    db.qual2 = pe ? s.d_rows + 3 * plane : nullptr;
    db.len2 = pe ? s.d_lens + e->max_batch : nullptr;
    // H2D of the text spans and records on the copy-in stream
    for (int m = 0; m < (pe ? 2 : 1); ++m) {
        HIP_TRY(e, hipMemcpyAsync(s.d_text[m], tb->text[m], tb->text_bytes[m], hipMemcpyHostToDevice, e->s_in));
        HIP_TRY(e, hipMemcpyAsync(s.d_trec[m], tb->rec[m], (size_t)tb->n * sizeof(fq_text_rec), hipMemcpyHostToDevice,
                                  e->s_in));
    }
    HIP_TRY(e, hipEventRecord(s.ev_in, e->s_in));
    HIP_TRY(e, hipStreamWaitEvent(e->stream, s.ev_in, 0));
    // planes from the text, the pack's kernels, then the output text
    for (int m = 0; m < (pe ? 2 : 1); ++m)
        HIP_TRY(e, fq_launch_text_tiles(s.d_text[m], s.d_trec[m], tb->n, tb->stride, const_cast<uint8_t*>(m ? db.seq2 : db.seq1),
                                        const_cast<uint8_t*>(m ? db.qual2 : db.qual1), const_cast<uint16_t*>(m ? db.len2 : db.len1),
                                        e->stream));
    HIP_TRY(e, hipMemsetAsync(s.d_err, 0, sizeof(int), e->stream));
    if ((rc = launch(e, db, s.d_res, e->stream, s.scratch, false, false, seq_no, s.d_err)) != FQ_OK) return rc;
    if ((rc = launch_text_out(e, s, tb->n)) != FQ_OK) return rc;
    HIP_TRY(e, hipEventRecord(s.ev_kern, e->stream));
    // D2H: records, output sizes and text (the text up to its input span: an upper bound of the
    // output, no device-to-host round trip for the exact size), the error word
    HIP_TRY(e, hipStreamWaitEvent(e->s_out, s.ev_kern, 0));
    const size_t nres = (size_t)tb->n * (pe ? 2 : 1);
    HIP_TRY(e, hipMemcpyAsync(results, s.d_res, nres * sizeof(fq_read_result), hipMemcpyDeviceToHost, e->s_out));
    HIP_TRY(e, hipMemcpyAsync(s.h_total, s.d_total, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, e->s_out));
    for (int m = 0; m < (mrg ? 1 : pe ? 2 : 1); ++m) {
        const size_t back = mrg ? merged_cap(tb->text_bytes[0], tb->text_bytes[1], (size_t)tb->n) : tb->text_bytes[m] + kTextSlack;
        HIP_TRY(e, hipMemcpyAsync(out->text[m], s.d_out[m], back, hipMemcpyDeviceToHost, e->s_out));
    }
    HIP_TRY(e, hipMemcpyAsync(s.h_err, s.d_err, sizeof(int), hipMemcpyDeviceToHost, e->s_out));
    HIP_TRY(e, hipEventRecord(s.ev_done, e->s_out));
    s.busy = true;
    s.text_out = out;
    e->pending.push_back(Pending{seq_no, k, false, 0});
    return FQ_OK;
}

// ---- raw FASTQ streams -----------------------------------------------------------------------

// the raw-window buffers of slot s (the text-pack buffers at raw capacity plus the line index)
static int ensure_raw(fq_engine* e, Slot& s) {
    if (s.raw_ready) return FQ_OK;
    const bool pe = e->p.paired;
    const size_t text = (size_t)e->raw_nblocks * 4096;
    const size_t recs = (size_t)e->max_batch + 1;
    const size_t cap_lines = 4 * recs + 8;
    for (int m = 0; m < 2; ++m) {
        if (s.d_text[m]) (void)hipFree(s.d_text[m]);
        if (s.d_out[m]) (void)hipFree(s.d_out[m]);
        if (s.d_trec[m]) (void)hipFree(s.d_trec[m]);
        if (s.d_tsize[m]) (void)hipFree(s.d_tsize[m]);
        if (s.d_toff[m]) (void)hipFree(s.d_toff[m]);
        s.d_text[m] = s.d_out[m] = nullptr;
        s.d_trec[m] = nullptr;
        s.d_tsize[m] = s.d_toff[m] = nullptr;
        for (uint32_t** q : {&s.d_lines[m], &s.d_bcnt[m], &s.d_bbase[m]})
            if (*q) {
                (void)hipFree(*q);
                *q = nullptr;
            }
        if (s.d_ad[m]) (void)hipFree(s.d_ad[m]);
        s.d_ad[m] = nullptr;
        if (m == 1 && !pe) continue;
        HIP_TRY(e, hipMalloc(&s.d_text[m], text));
        // (+ the adapter entries' slack; -m: mate 0's takes the merged stream of both mates' text)
        const size_t out = pe && m == 0 && e->p.merge_enabled ? merged_cap(text, text, recs) + 3 * recs + 64 : text + 4 * recs + 64;
        HIP_TRY(e, hipMalloc(&s.d_out[m], out));
        HIP_TRY(e, hipMalloc(&s.d_trec[m], recs * sizeof(fq_text_rec)));
        HIP_TRY(e, hipMalloc(&s.d_tsize[m], recs * sizeof(uint32_t)));
        HIP_TRY(e, hipMalloc(&s.d_toff[m], recs * sizeof(uint32_t)));
        HIP_TRY(e, hipMalloc(&s.d_lines[m], cap_lines * sizeof(uint32_t)));
        HIP_TRY(e, hipMalloc(&s.d_bcnt[m], (size_t)e->raw_nblocks * sizeof(uint32_t)));
        HIP_TRY(e, hipMalloc(&s.d_bbase[m], (size_t)e->raw_nblocks * sizeof(uint32_t)));

    }
    s.text_cap[0] = s.text_cap[1] = 0;  // (not the text-pack sizes: ensure_text re-allocates)
    s.trec_cap = 0;
    if (s.d_scan) (void)hipFree(s.d_scan);
    s.scan_bytes = std::max(fq_raw_scan_temp_bytes((int)e->raw_nblocks, (int)recs), fq_text_scan_temp_bytes((int)recs));
    HIP_TRY(e, hipMalloc(&s.d_scan, s.scan_bytes));
    if (!s.d_total) HIP_TRY(e, hipMalloc(&s.d_total, 4 * sizeof(unsigned long long)));
    if (!s.h_total) HIP_TRY(e, hipHostMalloc((void**)&s.h_total, 4 * sizeof(unsigned long long), hipHostMallocDefault));
    if (!s.d_rstate) HIP_TRY(e, hipMalloc(&s.d_rstate, 2 * sizeof(fq_raw_state)));
    if (!s.h_rstate) HIP_TRY(e, hipHostMalloc((void**)&s.h_rstate, 2 * sizeof(fq_raw_state), hipHostMallocDefault));
    if (!s.ev_idx) HIP_TRY(e, hipEventCreateWithFlags(&s.ev_idx, hipEventDisableTiming));
    s.raw_ready = true;
    return FQ_OK;
}

int fq_engine_raw_begin(fq_engine* e, uint64_t window_cap, uint64_t carry_cap) {
    if (!e) return FQ_E_INVALID;
    if (!e->pending.empty() || !e->raw_queued.empty()) return fail(e, FQ_E_INVALID, "fq_engine_raw_begin with packs in flight");
    if (e->p.correction_enabled || e->p.umi_front1 > 0 || e->p.umi_front2 > 0 ||
        (e->p.merge_enabled && e->p.discard_unmerged))
        return fail(e, FQ_E_INVALID, "raw streams take no -c, UMI or --discard_unmerged options");
    const double tb = engine_timing() ? now_s() : 0;
    struct Stamp {
        double t;
        ~Stamp() {
            if (t > 0) std::fprintf(stderr, "fq_engine_raw_begin: %.2f ms\n", 1e3 * (now_s() - t));
        }
    } stamp{tb};
    carry_cap = (carry_cap + 4095) / 4096 * 4096;
    if (!window_cap || carry_cap + window_cap + 4096 >= (1ull << 31) || e->max_batch <= 0)
        return fail(e, FQ_E_INVALID, "raw window / carry capacity out of range");
    HIP_TRY(e, hipSetDevice(e->device));
    HIP_TRY(e, hipDeviceSynchronize());
    if (!e->s_idx) HIP_TRY(e, hipStreamCreateWithFlags(&e->s_idx, hipStreamNonBlocking));
    const uint32_t nb = (uint32_t)((carry_cap + window_cap + 64 + 4095) / 4096);
    if (!e->raw || nb != e->raw_nblocks || carry_cap != e->raw_ccap)
        for (Slot& s : e->slots) s.raw_ready = false;
    e->raw = true;
    e->raw_wcap = window_cap;
    e->raw_ccap = carry_cap;
    e->raw_nblocks = nb;
    e->raw_prev_slot = -1;
    e->raw_queued.clear();
    return FQ_OK;
}

int fq_engine_raw_enqueue(fq_engine* e, const fq_raw_window* w) {
    if (!e || !w) return FQ_E_INVALID;
    if (!e->raw) return fail(e, FQ_E_INVALID, "fq_engine_raw_enqueue before fq_engine_raw_begin");
    if (e->raw_queued.size() >= 3) return fail(e, FQ_E_INVALID, "three raw windows are already waiting for fq_engine_raw_launch");
    const bool pe = e->p.paired;
    for (int m = 0; m < (pe ? 2 : 1); ++m)
        if (w->n[m] > e->raw_wcap || (w->n[m] && !w->bytes[m])) return fail(e, FQ_E_INVALID, "raw window exceeds its capacity");
    HIP_TRY(e, hipSetDevice(e->device));
    const int k = (e->raw_prev_slot + 1) % kRawSlots;
    int rc = retire_slot(e, k);
    if (rc != FQ_OK) return rc;
    Slot& s = e->slots[k];
    const bool fresh = !s.raw_ready;
    const double ts = fresh && engine_timing() ? now_s() : 0;
    if ((rc = alloc_slot(e, s)) != FQ_OK) return rc;
    if ((rc = ensure_raw(e, s)) != FQ_OK) return rc;
    if (ts > 0) std::fprintf(stderr, "fq_engine_raw_enqueue: slot %d set up in %.2f ms\n", k, 1e3 * (now_s() - ts));
    {
        LinkChain& lc = link_chain(e->device);
        std::lock_guard<std::mutex> g(lc.m);
        if (lc.in && lc.in_owner != e) HIP_TRY(e, hipStreamWaitEvent(e->s_in, lc.in, 0));
        for (int m = 0; m < (pe ? 2 : 1); ++m)
            if (w->n[m])
                HIP_TRY(e, hipMemcpyAsync(s.d_text[m] + e->raw_ccap, w->bytes[m], w->n[m], hipMemcpyHostToDevice, e->s_in));
        HIP_TRY(e, hipEventRecord(s.ev_in, e->s_in));
        lc.in = s.ev_in, lc.in_owner = e;
    }
    HIP_TRY(e, hipStreamWaitEvent(e->s_idx, s.ev_in, 0));
    s.raw_n[0] = w->n[0];
    s.raw_n[1] = pe ? w->n[1] : 0;
    fq_raw_text_args a{};
    const Slot* ps = e->raw_prev_slot >= 0 ? &e->slots[e->raw_prev_slot] : nullptr;
    for (int m = 0; m < 2; ++m) {
        a.text[m] = s.d_text[m];
        a.prev_text[m] = ps ? ps->d_text[m] : nullptr;
        a.raw_bytes[m] = (uint32_t)w->n[m];
        a.bcnt[m] = s.d_bcnt[m];
        a.bbase[m] = s.d_bbase[m];
        a.lines[m] = s.d_lines[m];
        a.rec[m] = s.d_trec[m];
    }
    a.prev_state = ps ? ps->d_rstate : nullptr;
    a.state = s.d_rstate;
    a.carry_cap = (uint32_t)e->raw_ccap;
    a.nblocks = e->raw_nblocks;
    a.cap_lines = (uint32_t)(4 * ((size_t)e->max_batch + 1) + 8);
    a.cap_records = e->max_batch + 1;
    a.max_len = std::min(e->max_stride, e->p.max_cycles);
    HIP_TRY(e, fq_launch_raw_index(a, pe ? 2 : 1, e->max_batch, s.d_scan, s.scan_bytes, e->s_idx));
    HIP_TRY(e, hipMemcpyAsync(s.h_rstate, s.d_rstate, 2 * sizeof(fq_raw_state), hipMemcpyDeviceToHost, e->s_idx));
    HIP_TRY(e, hipEventRecord(s.ev_idx, e->s_idx));
    e->raw_queued.push_back(k);
    e->raw_prev_slot = k;
    return FQ_OK;
}

// the oldest enqueued window's index, once its copy back has landed
static void raw_result_of(const fq_engine* e, const Slot& s, fq_raw_result* r) {
    const int mates = e->p.paired ? 2 : 1;
    std::memset(r, 0, sizeof *r);
    const int n = s.h_rstate[0].n;
    r->pairs = n;
    for (int m = 0; m < mates; ++m) {
        const fq_raw_state& st = s.h_rstate[m];
        // (after an overflow every byte of the carry and the window is still to be read)
        r->carry[m] = st.overflow ? (uint64_t)st.carry_in + s.raw_n[m] : (uint64_t)(st.avail - st.consumed);
        r->text_bytes[m] = st.consumed;
        r->max_len = std::max(r->max_len, st.max_len);
        if (st.overflow || st.first_bad == n) r->stop = 1;
    }
}

int fq_engine_raw_wait(fq_engine* e, fq_raw_result* r) {
    if (!e) return FQ_E_INVALID;
    if (e->raw_queued.empty()) return fail(e, FQ_E_INVALID, "fq_engine_raw_wait without an enqueued window");
    HIP_TRY(e, hipSetDevice(e->device));
    const Slot& s = e->slots[e->raw_queued.front()];
    HIP_TRY(e, hipEventSynchronize(s.ev_idx));
    if (r) raw_result_of(e, s, r);
    return FQ_OK;
}

int fq_engine_raw_launch(fq_engine* e, fq_raw_result* r, fq_raw_out* out, uint64_t seq_no) {
    if (!e || !r || !out) return FQ_E_INVALID;
    if (e->raw_queued.empty()) return fail(e, FQ_E_INVALID, "fq_engine_raw_launch without an enqueued window");
    HIP_TRY(e, hipSetDevice(e->device));
    const int k = e->raw_queued.front();
    e->raw_queued.pop_front();
    Slot& s = e->slots[k];
    HIP_TRY(e, hipEventSynchronize(s.ev_idx));  // (returns at once after fq_engine_raw_wait)
    const bool pe = e->p.paired;
    const int mates = pe ? 2 : 1;
    raw_result_of(e, s, r);
    const int n = r->pairs;
    out->text.bytes[0] = out->text.bytes[1] = 0;
    out->adapter_bytes[0] = out->adapter_bytes[1] = 0;
    if (n <= 0) {
        e->pending.push_back(Pending{seq_no, -1, true, 0});
        return FQ_OK;
    }
    const bool recs_only = out->results != nullptr;  // (records-only egress: the caller formats)
    for (int m = 0; m < mates; ++m)
        if (recs_only ? !out->rec[m] : !out->text.text[m]) return fail(e, FQ_E_INVALID, "raw pack: missing output buffer");
    const size_t plane = fq_batch_bytes(e->max_batch, e->max_stride);
    fq_batch db{};
    db.n = n;
    db.stride = std::max(16, (r->max_len + 15) & ~15);
    db.seq1 = s.d_rows;
    db.qual1 = s.d_rows + plane;
    db.len1 = s.d_lens;
    db.seq2 = pe ? s.d_rows + 2 * plane : nullptr;
    db.qual2 = pe ? s.d_rows + 3 * plane : nullptr;
    db.len2 = pe ? s.d_lens + e->max_batch : nullptr;
    HIP_TRY(e, hipStreamWaitEvent(e->stream, s.ev_idx, 0));
    for (int m = 0; m < mates; ++m)
        HIP_TRY(e, fq_launch_text_tiles(s.d_text[m], s.d_trec[m], n, db.stride, const_cast<uint8_t*>(m ? db.seq2 : db.seq1),
                                        const_cast<uint8_t*>(m ? db.qual2 : db.qual1), const_cast<uint16_t*>(m ? db.len2 : db.len1),
                                        e->stream));
    HIP_TRY(e, hipMemsetAsync(s.d_err, 0, sizeof(int), e->stream));
    int rc = launch(e, db, s.d_res, e->stream, s.scratch, false, false, seq_no, s.d_err);
    if (rc != FQ_OK) return rc;
    HIP_TRY(e, hipMemsetAsync(s.d_total, 0, 4 * sizeof(unsigned long long), e->stream));
    if (recs_only) {  // the records and their line offsets back, no output text
        HIP_TRY(e, hipEventRecord(s.ev_kern, e->stream));
        HIP_TRY(e, hipStreamWaitEvent(e->s_out, s.ev_kern, 0));
        HIP_TRY(e, hipMemcpyAsync(out->results, s.d_res, (size_t)n * mates * sizeof(fq_read_result), hipMemcpyDeviceToHost,
                                  e->s_out));
        for (int m = 0; m < mates; ++m)
            HIP_TRY(e, hipMemcpyAsync(out->rec[m], s.d_trec[m], (size_t)n * sizeof(fq_text_rec), hipMemcpyDeviceToHost, e->s_out));
        HIP_TRY(e, hipMemcpyAsync(s.h_total, s.d_total, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, e->s_out));
        HIP_TRY(e, hipMemcpyAsync(s.h_err, s.d_err, sizeof(int), hipMemcpyDeviceToHost, e->s_out));
        HIP_TRY(e, hipEventRecord(s.ev_done, e->s_out));
        s.busy = true;
        s.text_out = &out->text;
        s.raw_out = out;
        e->pending.push_back(Pending{seq_no, k, false, 0});
        return FQ_OK;
    }
    // each mate's copy back: its output text (<= the input it spans) and the adapter entries after
    // it (per record, output + entry <= input + 3 bytes)
    // (-m: mate 0's output is the merged stream, mate 1's is empty: only its adapter entries)
    const bool mrg = pe && e->p.merge_enabled;
    size_t back[2] = {0, 0};
    for (int m = 0; m < mates; ++m) back[m] = (size_t)r->text_bytes[m] + kTextSlack + 3 * (size_t)n;
    if (mrg) back[0] = merged_cap(r->text_bytes[0], r->text_bytes[1], (size_t)n) + 3 * (size_t)n;
    if ((rc = launch_text_out(e, s, n)) != FQ_OK) return rc;
    for (int m = 0; m < mates; ++m) {
        if (e->p.adapter_trimming)
            HIP_TRY(e, fq_launch_raw_adapters(s.d_text[m], s.d_trec[m], s.d_res, n, pe ? 1 : 0, m, s.d_tsize[m], s.d_toff[m],
                                              s.d_scan, s.scan_bytes, s.d_out[m], s.d_total + m, back[m], s.d_total + 2 + m,
                                              e->stream));
    }
    // the output sizes (and the error word) behind the kernels; the text follows once they are in
    HIP_TRY(e, hipMemcpyAsync(s.h_total, s.d_total, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(e, hipMemcpyAsync(s.h_err, s.d_err, sizeof(int), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(e, hipEventRecord(s.ev_kern, e->stream));
    for (int m = 0; m < 2; ++m) {
        s.copy_dst[m] = m < mates ? out->text.text[m] : nullptr;
        s.copy_cap[m] = m < mates ? back[m] : 0;
    }
    s.copy_pending = true;
    s.busy = true;
    s.text_out = &out->text;
    s.raw_out = out;
    e->pending.push_back(Pending{seq_no, k, false, 0});
    return issue_copies(e, -1);
}

int fq_engine_raw_end(fq_engine* e) {
    if (!e) return FQ_E_INVALID;
    if (!e->raw) return FQ_OK;
    HIP_TRY(e, hipSetDevice(e->device));
    if (e->s_idx) HIP_TRY(e, hipStreamSynchronize(e->s_idx));  // (the index stream waits for the copies)
    e->raw_queued.clear();
    e->raw_prev_slot = -1;
    e->raw = false;
    return FQ_OK;
}

int fq_host_register(const void* p, size_t bytes) {
    if (!p || !bytes) return FQ_E_INVALID;
    return hipHostRegister(const_cast<void*>(p), bytes, hipHostRegisterReadOnly) == hipSuccess ? FQ_OK : FQ_E_HIP;
}

int fq_host_unregister(const void* p) {
    if (!p) return FQ_E_INVALID;
    return hipHostUnregister(const_cast<void*>(p)) == hipSuccess ? FQ_OK : FQ_E_HIP;
}

int fq_engine_poll(fq_engine* e, int wait, uint64_t* seq_no) {
    if (!e) return FQ_E_INVALID;
    if (e->pending.empty()) return 0;
    HIP_TRY(e, hipSetDevice(e->device));
    int rc0 = issue_copies(e, -1);  // (raw packs whose sizes are in: their copies back start now)
    if (rc0 != FQ_OK) return rc0;
    Pending& q = e->pending.front();
    if (!q.done) {
        Slot& s = e->slots[q.slot];
        if (s.copy_pending && !wait) return 0;
        if (!wait) {
            const hipError_t st = hipEventQuery(s.ev_done);
            if (st == hipErrorNotReady) return 0;
            if (st != hipSuccess) return hip_fail(e, st, "hipEventQuery");
        }
        int rc = retire_slot(e, q.slot);
        if (rc != FQ_OK) return rc;
    }
    const Pending done = q;
    e->pending.pop_front();
    if (seq_no) *seq_no = done.seq_no;
    if (done.err) return fail(e, FQ_E_TOO_LONG, "a read is longer than max_cycles or the row stride");
    return 1;
}

int fq_engine_pending(const fq_engine* e) { return e ? (int)e->pending.size() : FQ_E_INVALID; }

int fq_engine_process(fq_engine* e, const fq_batch* hb, fq_read_result* results) {
    if (!e || !hb || !results) return FQ_E_INVALID;
    if (!e->pending.empty()) return fail(e, FQ_E_INVALID, "fq_engine_process with submitted packs not yet polled");
    int rc = fq_engine_submit(e, hb, results, 0);
    if (rc != FQ_OK) return rc;
    rc = fq_engine_poll(e, 1, nullptr);
    return rc == 1 ? FQ_OK : rc;
}

int fq_engine_process_device(fq_engine* e, const fq_batch* db, fq_read_result* dres, void* stream) {
    if (!e || !db) return FQ_E_INVALID;
    if (db->n < 0 || db->stride <= 0 || (db->stride & 15) || !db->seq1 || !db->qual1 || !db->len1 ||
        (e->p.paired && (!db->seq2 || !db->qual2 || !db->len2)))
        return fail(e, FQ_E_INVALID, "bad device batch");
    if (e->p.correction_enabled && db->stride > 32768)
        return fail(e, FQ_E_INVALID, "-c takes reads of at most 32767 bases (the record's overlap offset is 16-bit)");
    HIP_TRY(e, hipSetDevice(e->device));
    // NULL is the HIP default stream
    return launch(e, *db, dres, (hipStream_t)stream, e->scratch, true, true, e->calls++, e->err);
}

size_t fq_engine_acc_words(const fq_engine* e) { return e ? e->acc_words : 0; }

int fq_engine_set_dup(fq_engine* e, fq_dup* d) {
    if (!e) return FQ_E_INVALID;
    if (d) {
        int dev = -1;
        if (fq_dup_device(d, &dev) != FQ_OK || dev != e->device)
            return fail(e, FQ_E_INVALID, "the duplication table is on another device");
    }
    HIP_TRY(e, hipSetDevice(e->device));
    HIP_TRY(e, hipDeviceSynchronize());  // packs in flight finish with the old table
    e->dup = d;
    return FQ_OK;
}

int fq_engine_acc_device_ptr(fq_engine* e, uint64_t** dptr) {
    if (!e || !dptr) return FQ_E_INVALID;
    *dptr = reinterpret_cast<uint64_t*>(e->acc);
    return FQ_OK;
}

int fq_engine_read_acc(fq_engine* e, uint64_t* host, size_t words) {
    if (!e || !host || words < e->acc_words) return FQ_E_INVALID;
    HIP_TRY(e, hipSetDevice(e->device));
    HIP_TRY(e, hipDeviceSynchronize());
    HIP_TRY(e, hipMemcpy(host, e->acc, e->acc_words * 8, hipMemcpyDeviceToHost));
    return check_err(e);
}

int fq_engine_set_acc_buffer(fq_engine* e, uint64_t* device_acc) {
    if (!e) return FQ_E_INVALID;
    e->acc = device_acc ? reinterpret_cast<unsigned long long*>(device_acc) : e->own_acc;
    return FQ_OK;
}

int fq_engine_reset_acc(fq_engine* e) {
    if (!e) return FQ_E_INVALID;
    HIP_TRY(e, hipSetDevice(e->device));
    HIP_TRY(e, hipMemsetAsync(e->acc, 0, e->acc_words * 8, e->stream));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    return FQ_OK;
}

int fq_engine_sync(fq_engine* e) {
    if (!e) return FQ_E_INVALID;
    HIP_TRY(e, hipSetDevice(e->device));
    const int rc = issue_copies(e, -2);  // (the copies back of every raw pack launched)
    if (rc != FQ_OK) return rc;
    HIP_TRY(e, hipDeviceSynchronize());
    return check_err(e);
}

const char* fq_engine_last_error(const fq_engine* e) { return e ? e->last_error.c_str() : g_create_error.c_str(); }

int fq_engine_device_info(const fq_engine* e, int* device, char* arch, size_t arch_len) {
    if (!e) return FQ_E_INVALID;
    if (device) *device = e->device;
    if (arch && arch_len) std::snprintf(arch, arch_len, "%s", e->arch);
    return FQ_OK;
}

// Page-locked host memory as anonymous transparent-huge-page memory, populated, then registered
// with every device (portable): 0.06 s per GiB to set up and 0.04 s to release, against 0.23 s
// and 0.13 s for hipHostMalloc (tools/micro/h2d.hip on MI355X), and DMA at the same 57 GB/s.
// The mapping length of each block is kept for fq_host_free; hipHostMalloc is the fallback.
namespace {
std::mutex g_host_mu;
std::unordered_map<void*, size_t> g_host_maps;  // registered anonymous mappings -> length
}  // namespace

int fq_host_alloc(size_t bytes, void** out) {
    if (!out) return FQ_E_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return FQ_E_NO_DEVICE;
    const size_t huge = (size_t)2 << 20;
    const size_t len = ((bytes ? bytes : 1) + huge - 1) / huge * huge;
    void* m = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m != MAP_FAILED) {
        (void)madvise(m, len, MADV_HUGEPAGE);
        std::memset(m, 0, len);  // populate (registration pins what is there)
        if (hipHostRegister(m, len, hipHostRegisterPortable) == hipSuccess) {
            std::lock_guard<std::mutex> g(g_host_mu);
            g_host_maps[m] = len;
            *out = m;
            return FQ_OK;
        }
        munmap(m, len);
    }
    if (hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocPortable) != hipSuccess) {
        *out = nullptr;
        return FQ_E_NOMEM;
    }
    return FQ_OK;
}

int fq_host_free(void* p) {
    if (!p) return FQ_OK;
    size_t len = 0;
    {
        std::lock_guard<std::mutex> g(g_host_mu);
        auto it = g_host_maps.find(p);
        if (it != g_host_maps.end()) {
            len = it->second;
            g_host_maps.erase(it);
        }
    }
    if (len) {
        const bool ok = hipHostUnregister(p) == hipSuccess;
        munmap(p, len);
        return ok ? FQ_OK : FQ_E_HIP;
    }
    return hipHostFree(p) == hipSuccess ? FQ_OK : FQ_E_HIP;
}

int fq_synth_fill_device(const fq_batch* db, uint64_t seed, uint64_t first_index, int32_t read_len, void* stream) {
    if (!db || read_len <= 0 || read_len > db->stride || !db->seq1 || !db->qual1 || !db->len1)
        return FQ_E_INVALID;
    hipError_t he = fq_launch_synth(*db, seed, first_index, read_len, (hipStream_t)stream);
    return he == hipSuccess ? FQ_OK : FQ_E_HIP;
}

double fq_engine_last_kernel_ms(const fq_engine* e) {
    if (!e || !e->timed) return 0.0;
    float ms = 0.f;
    if (hipEventSynchronize(e->ev1) != hipSuccess) return 0.0;
    if (hipEventElapsedTime(&ms, e->ev0, e->ev1) != hipSuccess) return 0.0;
    return ms;
}

}  // extern "C"
