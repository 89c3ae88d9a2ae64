// cpu_engine.cpp -- TEST INFRASTRUCTURE ONLY: a CPU stand-in for the engine's host-facing C-ABI
// (include/fqengine.h), built on the oracle (fq_oracle.c), so the tool's host pipeline
// (fqtool_amd/host: reader, one dispatcher per engine, formatter, writers, pool, and the raw stream's
// window reader, per-engine threads and ordered enqueue/launch hand-offs) runs without a GPU under
// ThreadSanitizer (`make tsan`, tests/test_tsan_cpu.py) and in the CPU suite (`make cpuhost`,
// tests/test_raw_cpu.py).  It is linked only into those builds under build/; the product
// (fqtool_amd/lib/libfqengine.so) never loads it.
//
// Each engine runs its work on a worker thread of its own, in call order, so the host sees the same
// asynchronous contract as the device pipeline: fq_engine_submit / _submit_text / _raw_enqueue /
// _raw_launch return at once, the host's batch, text and window bytes are read and its `results` and
// output buffers written later, fq_engine_poll reports packs in order (and only then sets the output
// sizes).  Text packs and raw streams restate text.hip (output text, the merged stream) and raw.hip
// (record cut, "plain" test, carry, stop) on the CPU.  Duplication tables do not merge across
// engines here (fq_dup_merge fails), so -d runs take one engine.
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <chrono>
#include <thread>
#include <vector>
#include <algorithm>
#include <climits>

#include "fq_oracle.h"

struct fq_dup {
    orc_dup* d;
};
struct fq_kmer_set {
    void* k;
};

struct RawWin;  // a raw window (below)

struct fq_engine {
    fq_params p;
    int max_batch = 0, max_stride = 0;
    std::vector<uint64_t> acc;
    fq_dup* dup = nullptr;
    std::string err;
    // work in call order on the worker thread: packs (reported by fq_engine_poll) and raw-window
    // indexing (not reported)
    struct Task {
        std::function<int(Task&)> fn;  // runs on the worker; returns FQ_OK or an FQ_E_* code
        uint64_t seq = 0;
        int rc = FQ_OK;
        bool done = false;
        bool pack = true;
        // output sizes, published to the caller's fq_text_out / fq_raw_out by fq_engine_poll
        fq_text_out* text_out = nullptr;
        fq_raw_out* raw_out = nullptr;
        uint64_t bytes[2] = {0, 0}, ad_bytes[2] = {0, 0};
        std::chrono::steady_clock::time_point ready_at{};  // (FQ_CPU_ENGINE_DELAY_US)
    };
    std::deque<std::shared_ptr<Task>> work;   // not yet run, in call order
    std::deque<std::shared_ptr<Task>> packs;  // submitted packs, in order; front = oldest not yet polled
    std::mutex m;
    std::condition_variable cv;
    bool stop = false;
    std::thread worker;
    // raw mode
    bool raw = false;
    uint64_t raw_wcap = 0, raw_ccap = 0;
    std::shared_ptr<RawWin> raw_prev;               // the last window enqueued
    std::deque<std::shared_ptr<RawWin>> raw_queued;  // enqueued, not launched

    // FQ_CPU_ENGINE_DELAY_US: a pack is reported done no earlier than this long after its submission
    // (its work still runs at once, so raw-window indexing is not held up behind it -- as on the GPU,
    // where the index runs on its own stream while earlier packs' kernels run).  Tests: packs stay in
    // flight, so the host's pack and staging budgets run out while engines wait for their turns.
    long delay_us = 0;
    void run() {
        std::unique_lock<std::mutex> lk(m);
        for (;;) {
            if (work.empty()) {
                if (stop) return;
                cv.wait(lk);
                continue;
            }
            std::shared_ptr<Task> t = work.front();
            work.pop_front();
            lk.unlock();
            const int rc = t->fn(*t);
            lk.lock();
            t->rc = rc;
            t->done = true;
            cv.notify_all();
        }
    }
    // queues fn; a pack is also reported by fq_engine_poll
    std::shared_ptr<Task> post(std::function<int(Task&)> fn, bool pack, uint64_t seq, fq_text_out* text_out = nullptr,
                               fq_raw_out* raw_out = nullptr) {
        auto t = std::make_shared<Task>();
        t->fn = std::move(fn);
        t->pack = pack;
        t->seq = seq;
        t->text_out = text_out;
        t->raw_out = raw_out;
        t->ready_at = std::chrono::steady_clock::now() + std::chrono::microseconds(pack ? delay_us : 0);
        std::lock_guard<std::mutex> lk(m);
        work.push_back(t);
        if (pack) packs.push_back(t);
        cv.notify_all();
        return t;
    }
    void wait(const std::shared_ptr<Task>& t) {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return t->done; });
    }
    // the pack's records into the accumulator (and the duplication table)
    int process(const fq_batch& b, fq_read_result* res) {
        std::vector<uint64_t> a(acc.size(), 0);
        const int rc = orc_process_batch(&p, &b, res, a.data());
        if (rc == FQ_OK && dup) orc_dup_add_batch(dup->d, &b, p.paired);
        std::lock_guard<std::mutex> lk(m);
        for (size_t i = 0; i < acc.size(); ++i) acc[i] += a[i];
        return rc;
    }
};

static int fail(fq_engine* e, int rc, const char* msg) {
    e->err = msg;
    return rc;
}

extern "C" {

int fq_engine_create(const fq_params* params, int device, int32_t max_batch, int32_t max_stride, fq_engine** out) {
    (void)device;
    if (!params || !out || max_batch < 0 || max_stride < 0 || (max_stride & 15)) return FQ_E_INVALID;
    fq_engine* e = new fq_engine();
    e->p = *params;
    e->max_batch = max_batch;
    e->max_stride = max_stride;
    e->acc.assign(fq_acc_words(params->insert_size_max, params->max_cycles), 0);
    if (const char* d = std::getenv("FQ_CPU_ENGINE_DELAY_US")) e->delay_us = std::atol(d);
    e->worker = std::thread([e] { e->run(); });
    *out = e;
    return FQ_OK;
}

int fq_engine_destroy(fq_engine* e) {
    if (!e) return FQ_E_INVALID;
    {
        std::lock_guard<std::mutex> lk(e->m);
        e->stop = true;
        e->cv.notify_all();
    }
    e->worker.join();
    delete e;
    return FQ_OK;
}

int fq_engine_submit(fq_engine* e, const fq_batch* b, fq_read_result* results, uint64_t seq_no) {
    if (!e || !b || !results) return FQ_E_INVALID;
    const fq_batch bb = *b;
    e->post([e, bb, results](fq_engine::Task&) { return e->process(bb, results); }, true, seq_no);
    return FQ_OK;
}

int fq_engine_poll(fq_engine* e, int wait, uint64_t* seq_no) {
    if (!e) return FQ_E_INVALID;
    std::unique_lock<std::mutex> lk(e->m);
    if (e->packs.empty()) return 0;
    if (!e->packs.front()->done || std::chrono::steady_clock::now() < e->packs.front()->ready_at) {
        if (!wait) return 0;
        e->cv.wait(lk, [e] { return e->packs.front()->done; });
        const auto at = e->packs.front()->ready_at;
        lk.unlock();
        std::this_thread::sleep_until(at);
        lk.lock();
    }
    const std::shared_ptr<fq_engine::Task> t = e->packs.front();
    e->packs.pop_front();
    if (seq_no) *seq_no = t->seq;
    if (t->rc != FQ_OK) return fail(e, t->rc, "oracle stand-in: the pack failed");
    // (as the device engine: a text / raw pack's output sizes are set when it is reported)
    if (t->text_out) {
        t->text_out->bytes[0] = t->bytes[0];
        t->text_out->bytes[1] = t->bytes[1];
    }
    if (t->raw_out) {
        t->raw_out->adapter_bytes[0] = t->ad_bytes[0];
        t->raw_out->adapter_bytes[1] = t->ad_bytes[1];
    }
    return 1;
}

int fq_engine_pending(const fq_engine* e) {
    if (!e) return FQ_E_INVALID;
    std::lock_guard<std::mutex> lk(const_cast<fq_engine*>(e)->m);
    return (int)e->packs.size();
}

int fq_engine_process(fq_engine* e, const fq_batch* b, fq_read_result* results) {
    int rc = fq_engine_submit(e, b, results, 0);
    if (rc != FQ_OK) return rc;
    rc = fq_engine_poll(e, 1, nullptr);
    return rc == 1 ? FQ_OK : rc;
}

int fq_engine_sync(fq_engine* e) {
    if (!e) return FQ_E_INVALID;
    std::unique_lock<std::mutex> lk(e->m);
    e->cv.wait(lk, [e] {
        if (!e->work.empty()) return false;
        for (const auto& t : e->packs)
            if (!t->done) return false;
        return true;
    });
    return FQ_OK;
}

size_t fq_engine_acc_words(const fq_engine* e) { return e ? e->acc.size() : 0; }

int fq_engine_read_acc(fq_engine* e, uint64_t* host_acc, size_t words) {
    if (!e || !host_acc || words < e->acc.size()) return FQ_E_INVALID;
    fq_engine_sync(e);
    std::lock_guard<std::mutex> lk(e->m);
    std::memcpy(host_acc, e->acc.data(), e->acc.size() * 8);
    return FQ_OK;
}

int fq_engine_reset_acc(fq_engine* e) {
    if (!e) return FQ_E_INVALID;
    fq_engine_sync(e);
    std::lock_guard<std::mutex> lk(e->m);
    std::fill(e->acc.begin(), e->acc.end(), 0);
    return FQ_OK;
}

const char* fq_engine_last_error(const fq_engine* e) { return e ? e->err.c_str() : "no engine"; }

}  // extern "C"

// ---- FASTQ-text packs (text.hip restated) ----

namespace {

bool passes(const fq_read_result& r) { return !(r.flags & (FQ_RF_NULL | FQ_RF_INDEX_FILTERED)) && r.code == FQ_PASS_FILTER; }

char comp_base(char c) {
    switch (c) {
        case 'A': case 'a': return 'T';
        case 'T': case 't': return 'A';
        case 'C': case 'c': return 'G';
        case 'G': case 'g': return 'C';
        default: return 'N';
    }
}

char* put_read(char* d, const char* text, const fq_text_rec& R, const fq_read_result& r) {
    std::memcpy(d, text + R.name_off, R.name_len);
    d += R.name_len;
    *d++ = '\n';
    std::memcpy(d, text + R.seq_off + r.start, r.len);
    d += r.len;
    *d++ = '\n';
    std::memcpy(d, text + R.strand_off, R.strand_len);
    d += R.strand_len;
    *d++ = '\n';
    std::memcpy(d, text + R.qual_off + r.start, r.len);
    d += r.len;
    *d++ = '\n';
    return d;
}

// A text pack's kernels on the CPU: the planes from the text (text_tile_kernel), the oracle, the
// output text (text_write_kernel / merge_write_kernel); bytes[m] = mate m's output text.
int run_text_pack(fq_engine* e, int n, int stride, const char* const text[2], const fq_text_rec* const rec[2],
                  fq_read_result* res, char* const out[2], uint64_t bytes[2]) {
    const bool pe = e->p.paired;
    const int mates = pe ? 2 : 1;
    const size_t plane = fq_batch_bytes(n, stride);
    std::vector<uint8_t> rows((size_t)2 * mates * plane, 0);
    std::vector<uint16_t> lens((size_t)mates * n);
    for (int m = 0; m < mates; ++m)
        for (int i = 0; i < n; ++i) {
            const fq_text_rec& R = rec[m][i];
            if (R.len > stride) return FQ_E_TOO_LONG;
            fq_batch_put_row(rows.data() + (2 * m) * plane, stride, i, reinterpret_cast<const uint8_t*>(text[m] + R.seq_off), R.len);
            fq_batch_put_row(rows.data() + (2 * m + 1) * plane, stride, i, reinterpret_cast<const uint8_t*>(text[m] + R.qual_off), R.len);
            lens[(size_t)m * n + i] = R.len;
        }
    fq_batch b{};
    b.n = n;
    b.stride = stride;
    b.seq1 = rows.data();
    b.qual1 = rows.data() + plane;
    b.len1 = lens.data();
    if (pe) {
        b.seq2 = rows.data() + 2 * plane;
        b.qual2 = rows.data() + 3 * plane;
        b.len2 = lens.data() + n;
    }
    const int rc = e->process(b, res);
    if (rc != FQ_OK) return rc;
    bytes[0] = bytes[1] = 0;
    if (pe && e->p.merge_enabled) {  // the merged stream into mate 0's buffer (merge_write_kernel)
        char* d = out[0];
        for (int i = 0; i < n; ++i) {
            const fq_read_result &a = res[2 * i], &bb = res[2 * i + 1];
            const bool nn = !(a.flags & (FQ_RF_NULL | FQ_RF_INDEX_FILTERED)) && !(bb.flags & FQ_RF_NULL);
            const bool mrg = nn && (a.flags & FQ_RF_MERGED);
            if (!nn || (!mrg && e->p.discard_unmerged)) continue;
            const fq_text_rec &R1 = rec[0][i], &R2 = rec[1][i];
            if (!mrg) {
                if (a.code == FQ_PASS_FILTER) d = put_read(d, text[0], R1, a);
                if (bb.code == FQ_PASS_FILTER) d = put_read(d, text[1], R2, bb);
                continue;
            }
            if (a.code != FQ_PASS_FILTER) continue;
            const int m1 = a.m_len1, m2 = a.m_len2;
            const char* nm = text[0] + R1.name_off;
            int sp = -1;
            for (int k = 0; k < R1.name_len; ++k)
                if (nm[k] == ' ') {
                    sp = k;
                    break;
                }
            if (sp >= 0) {
                std::memcpy(d, nm, sp - 1);  // (the reference drops the byte before the space)
                d += sp - 1;
            }
            const std::string tag = "_merged_" + std::to_string(m1) + "_" + std::to_string(m2);
            std::memcpy(d, tag.data(), tag.size());
            d += tag.size();
            if (sp >= 0) {
                std::memcpy(d, nm + sp, R1.name_len - sp);
                d += R1.name_len - sp;
            }
            *d++ = '\n';
            const char* s1 = text[0] + R1.seq_off + a.start;
            const char* s2 = text[1] + R2.seq_off + bb.start;
            std::memcpy(d, s1, m1);
            d += m1;
            for (int j = 0; j < m2; ++j) d[j] = comp_base(s2[m2 - 1 - j]);
            d += m2;
            *d++ = '\n';
            std::memcpy(d, text[0] + R1.strand_off, R1.strand_len);
            d += R1.strand_len;
            *d++ = '\n';
            const char* q1 = text[0] + R1.qual_off + a.start;
            const char* q2 = text[1] + R2.qual_off + bb.start;
            std::memcpy(d, q1, m1);
            d += m1;
            for (int j = 0; j < m2; ++j) d[j] = q2[m2 - 1 - j];
            d += m2;
            *d++ = '\n';
        }
        bytes[0] = (uint64_t)(d - out[0]);
        return FQ_OK;
    }
    for (int m = 0; m < mates; ++m) {  // text_size_kernel / text_write_kernel
        char* d = out[m];
        for (int i = 0; i < n; ++i) {
            const bool ok = pe ? passes(res[2 * i]) && passes(res[2 * i + 1]) : passes(res[i]);
            if (ok) d = put_read(d, text[m], rec[m][i], res[pe ? 2 * i + m : i]);
        }
        bytes[m] = (uint64_t)(d - out[m]);
    }
    return FQ_OK;
}

bool text_options_ok(const fq_params& p) {
    return !(p.correction_enabled || p.umi_front1 > 0 || p.umi_front2 > 0 || (p.merge_enabled && p.discard_unmerged));
}

}  // namespace

// ---- raw FASTQ streams (raw.hip restated) ----

struct RawWin {
    std::shared_ptr<RawWin> prev;  // the window before (its unconsumed bytes are carried in)
    const char* src[2] = {nullptr, nullptr};
    uint64_t nraw[2] = {0, 0};
    std::unique_ptr<char[]> buf[2];  // [.. | carry | window] with the window at the carry capacity (uninitialised)
    uint32_t text_start[2] = {0, 0}, avail[2] = {0, 0}, carry_in[2] = {0, 0}, consumed[2] = {0, 0};
    bool overflow[2] = {false, false};
    int first_bad[2] = {INT32_MAX, INT32_MAX}, complete[2] = {0, 0};
    int max_len = 0, n = 0;
    std::vector<uint32_t> lines[2];
    std::vector<fq_text_rec> rec[2];
    std::shared_ptr<fq_engine::Task> indexed;  // the indexing task
};

namespace {

// raw_carry / raw_count / raw_lines / raw_records / raw_pair kernels of one window, in order after the
// previous window's (the worker runs tasks in call order)
void index_window(const fq_engine* e, RawWin& w) {
    const int mates = e->p.paired ? 2 : 1;
    const uint32_t ccap = (uint32_t)e->raw_ccap;
    const size_t cap_lines = 4 * ((size_t)e->max_batch + 1) + 8;
    const int cap_records = e->max_batch + 1;
    const int max_len = std::min(e->max_stride, e->p.max_cycles);
    for (int m = 0; m < mates; ++m) {
        const RawWin* ps = w.prev.get();
        const uint32_t carry = ps ? ps->avail[m] - ps->consumed[m] : 0u;
        const bool over = carry > ccap || (ps && ps->overflow[m]);
        w.text_start[m] = ccap - (over ? 0u : carry);
        w.carry_in[m] = carry;
        w.avail[m] = over ? 0u : carry + (uint32_t)w.nraw[m];
        w.overflow[m] = over;
        w.buf[m].reset(new char[(size_t)ccap + w.nraw[m] + 64]);
        if (ps && carry && !over) std::memcpy(w.buf[m].get() + (ccap - carry), ps->buf[m].get() + ps->text_start[m] + ps->consumed[m], carry);
        if (w.nraw[m]) std::memcpy(w.buf[m].get() + ccap, w.src[m], w.nraw[m]);
        const char* t = w.buf[m].get();
        const uint32_t lo = w.text_start[m], hi = lo + w.avail[m];
        std::vector<uint32_t>& L = w.lines[m];
        L.clear();
        for (uint32_t o = lo; o < hi && L.size() < cap_lines; ++o)
            if (t[o] == '\n' || t[o] == '\r') L.push_back(o);
        const int complete = std::min((int)(L.size() / 4), cap_records);
        w.complete[m] = complete;
        w.rec[m].assign((size_t)complete, fq_text_rec{});
        for (int i = 0; i < complete; ++i) {
            const uint32_t x = i ? L[4 * i - 1] + 1u : lo;
            const uint32_t t0 = L[4 * i], t1 = L[4 * i + 1], t2 = L[4 * i + 2], t3 = L[4 * i + 3];
            const uint32_t name_len = t0 - x, len = t1 - t0 - 1u, strand_len = t2 - t1 - 1u;
            const bool plain = t0 > x && t1 > t0 + 1u && t2 > t1 + 1u && t3 > t2 + 1u && t[x] == '@' && t[t0] == '\n' &&
                               t[t1] == '\n' && t[t2] == '\n' && t[t3] == '\n' && t3 - t2 == t1 - t0 &&
                               name_len <= 65535u && strand_len <= 65535u && len <= (uint32_t)max_len;
            if (!plain) {
                w.first_bad[m] = std::min(w.first_bad[m], i);
                continue;
            }
            fq_text_rec& r = w.rec[m][i];
            r.name_off = x;
            r.seq_off = t0 + 1u;
            r.strand_off = t1 + 1u;
            r.qual_off = t2 + 1u;
            r.name_len = (uint16_t)name_len;
            r.strand_len = (uint16_t)strand_len;
            r.len = (uint16_t)len;
            r.pad = 0;
            w.max_len = std::max(w.max_len, (int)len);
        }
    }
    int n = e->max_batch;
    for (int m = 0; m < mates; ++m) n = std::min(n, w.overflow[m] ? 0 : std::min(w.first_bad[m], w.complete[m]));
    w.n = n;
    for (int m = 0; m < mates; ++m) w.consumed[m] = n ? w.lines[m][4 * n - 1] + 1u - w.text_start[m] : 0u;
}

// trimmed-adapter entries of mate m after its output text (raw_ad_size / raw_ad_write kernels);
// returns the entries' bytes, or ~0 when they would not fit the copy back
uint64_t adapter_entries(const char* text, const fq_text_rec* rec, const fq_read_result* res, int n, bool pe, int m,
                         char* out, uint64_t base, uint64_t cap) {
    uint64_t total = 0;
    for (int i = 0; i < n; ++i) {
        const fq_read_result& r = res[pe ? 2 * i + m : i];
        if (!(r.flags & (FQ_RF_AD_OVERLAP | FQ_RF_AD_SEQ)) || r.ad_len == 0) continue;
        total += (r.flags & FQ_RF_AD_NEG) ? 5u : 3u + r.ad_len;
    }
    if (base + total > cap) return ~0ull;
    char* d = out + base;
    for (int i = 0; i < n; ++i) {
        const fq_read_result& r = res[pe ? 2 * i + m : i];
        if (!(r.flags & (FQ_RF_AD_OVERLAP | FQ_RF_AD_SEQ)) || r.ad_len == 0) continue;
        d[0] = (char)(r.ad_len & 0xFF);
        d[1] = (char)(r.ad_len >> 8);
        if (r.flags & FQ_RF_AD_NEG) {
            d[2] = 1;
            d[3] = (char)(r.ad_pos & 0xFF);
            d[4] = (char)(r.ad_pos >> 8);
            d += 5;
            continue;
        }
        d[2] = 0;
        std::memcpy(d + 3, text + rec[i].seq_off + r.ad_pos, r.ad_len);
        d += 3 + r.ad_len;
    }
    return total;
}

}  // namespace

extern "C" {

int fq_engine_submit_text(fq_engine* e, const fq_text_batch* tb, fq_read_result* results, fq_text_out* out,
                          uint64_t seq_no) {
    if (!e || !tb || !results || !out) return FQ_E_INVALID;
    const bool pe = e->p.paired;
    if (tb->n < 0 || tb->n > e->max_batch || tb->stride <= 0 || tb->stride > e->max_stride || (tb->stride & 15))
        return fail(e, FQ_E_INVALID, "text pack exceeds the engine's max_batch/max_stride (or stride % 16 != 0)");
    if (!text_options_ok(e->p)) return fail(e, FQ_E_INVALID, "text packs take no -c, UMI or --discard_unmerged options");
    for (int m = 0; m < (pe ? 2 : 1); ++m)
        if (tb->n > 0 && (!tb->text[m] || !tb->rec[m] || !out->text[m])) return fail(e, FQ_E_INVALID, "missing text pack arrays");
    out->bytes[0] = out->bytes[1] = 0;
    const fq_text_batch b = *tb;
    e->post(
        [e, b, results, out](fq_engine::Task& t) {
            char* const o[2] = {out->text[0], out->text[1]};
            return b.n ? run_text_pack(e, b.n, b.stride, b.text, b.rec, results, o, t.bytes) : FQ_OK;
        },
        true, seq_no, out);
    return FQ_OK;
}

int fq_engine_raw_begin(fq_engine* e, uint64_t window_cap, uint64_t carry_cap) {
    if (!e) return FQ_E_INVALID;
    {
        std::lock_guard<std::mutex> lk(e->m);
        if (!e->packs.empty() || !e->raw_queued.empty()) return fail(e, FQ_E_INVALID, "fq_engine_raw_begin with packs in flight");
    }
    if (!text_options_ok(e->p)) return fail(e, FQ_E_INVALID, "raw streams take no -c, UMI or --discard_unmerged options");
    carry_cap = (carry_cap + 4095) / 4096 * 4096;
    if (!window_cap || carry_cap + window_cap + 4096 >= (1ull << 31) || e->max_batch <= 0)
        return fail(e, FQ_E_INVALID, "raw window / carry capacity out of range");
    e->raw = true;
    e->raw_wcap = window_cap;
    e->raw_ccap = carry_cap;
    e->raw_prev.reset();
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
    auto win = std::make_shared<RawWin>();
    win->prev = e->raw_prev;
    for (int m = 0; m < (pe ? 2 : 1); ++m) {
        win->src[m] = w->bytes[m];
        win->nraw[m] = w->n[m];
    }
    // (the window's host bytes are read later, on the worker, as the device's copy is asynchronous)
    RawWin* wp = win.get();
    win->indexed = e->post(
        [e, wp](fq_engine::Task&) {
            index_window(e, *wp);
            wp->prev.reset();  // (only its carry was needed)
            return FQ_OK;
        },
        false, 0);
    e->raw_queued.push_back(win);
    e->raw_prev = win;
    return FQ_OK;
}

static void raw_result_of(const fq_engine* e, const RawWin& w, fq_raw_result* r) {
    std::memset(r, 0, sizeof *r);
    r->pairs = w.n;
    r->max_len = w.max_len;
    for (int m = 0; m < (e->p.paired ? 2 : 1); ++m) {
        r->carry[m] = w.overflow[m] ? (uint64_t)w.carry_in[m] + w.nraw[m] : (uint64_t)(w.avail[m] - w.consumed[m]);
        r->text_bytes[m] = w.consumed[m];
        if (w.overflow[m] || w.first_bad[m] == w.n) r->stop = 1;
    }
}

int fq_engine_raw_wait(fq_engine* e, fq_raw_result* r) {
    if (!e) return FQ_E_INVALID;
    if (e->raw_queued.empty()) return fail(e, FQ_E_INVALID, "fq_engine_raw_wait without an enqueued window");
    const std::shared_ptr<RawWin> w = e->raw_queued.front();
    e->wait(w->indexed);
    if (r) raw_result_of(e, *w, r);
    return FQ_OK;
}

int fq_engine_raw_launch(fq_engine* e, fq_raw_result* r, fq_raw_out* out, uint64_t seq_no) {
    if (!e || !r || !out) return FQ_E_INVALID;
    if (e->raw_queued.empty()) return fail(e, FQ_E_INVALID, "fq_engine_raw_launch without an enqueued window");
    std::shared_ptr<RawWin> w = e->raw_queued.front();
    e->raw_queued.pop_front();
    e->wait(w->indexed);  // (the window's index: waits as the device's launch does)
    const bool pe = e->p.paired;
    const int mates = pe ? 2 : 1;
    raw_result_of(e, *w, r);
    const int n = w->n;
    out->text.bytes[0] = out->text.bytes[1] = 0;
    out->adapter_bytes[0] = out->adapter_bytes[1] = 0;
    if (n <= 0) {
        e->post([](fq_engine::Task&) { return FQ_OK; }, true, seq_no);
        return FQ_OK;
    }
    const bool recs_only = out->results != nullptr;
    for (int m = 0; m < mates; ++m)
        if (recs_only ? !out->rec[m] : !out->text.text[m]) return fail(e, FQ_E_INVALID, "raw pack: missing output buffer");
    const int stride = std::max(16, (r->max_len + 15) & ~15);
    const uint64_t tb0 = r->text_bytes[0], tb1 = r->text_bytes[1];
    e->post(
        [e, w, out, n, stride, recs_only, pe, mates, tb0, tb1](fq_engine::Task& t) {
            std::vector<fq_read_result> res((size_t)n * mates);
            const char* text[2] = {w->buf[0].get(), pe ? w->buf[1].get() : nullptr};
            const fq_text_rec* rec[2] = {w->rec[0].data(), pe ? w->rec[1].data() : nullptr};
            if (recs_only) {  // the records and their line offsets, no output text
                std::vector<char> sink[2];
                for (int m = 0; m < mates; ++m) sink[m].resize((m ? tb1 : tb0) + (size_t)n * 28 + 64);
                char* const o[2] = {sink[0].data(), pe ? sink[1].data() : nullptr};
                uint64_t bytes[2];
                const int rc = run_text_pack(e, n, stride, text, rec, out->results, o, bytes);
                for (int m = 0; m < mates; ++m) std::memcpy(out->rec[m], rec[m], (size_t)n * sizeof(fq_text_rec));
                return rc;
            }
            char* const o[2] = {out->text.text[0], pe ? out->text.text[1] : nullptr};
            uint64_t bytes[2] = {0, 0};
            int rc = run_text_pack(e, n, stride, text, rec, res.data(), o, bytes);
            if (rc != FQ_OK) return rc;
            // the copies back: output text + adapter entries within text_bytes + 16 + 3n (-m: the
            // merged stream's capacity + 3n)
            uint64_t back[2];
            for (int m = 0; m < mates; ++m) back[m] = (m ? tb1 : tb0) + 16 + 3 * (uint64_t)n;
            if (pe && e->p.merge_enabled) back[0] = tb0 + tb1 + 24 * (uint64_t)n + 16 + 3 * (uint64_t)n;
            uint64_t ad[2] = {0, 0};
            for (int m = 0; m < mates; ++m)
                if (e->p.adapter_trimming) {
                    ad[m] = adapter_entries(text[m], rec[m], res.data(), n, pe, m, o[m], bytes[m], back[m]);
                    if (ad[m] == ~0ull) return (int)FQ_E_INVALID;
                }
            t.bytes[0] = bytes[0];
            t.bytes[1] = bytes[1];
            t.ad_bytes[0] = ad[0];
            t.ad_bytes[1] = ad[1];
            return FQ_OK;
        },
        true, seq_no, recs_only ? nullptr : &out->text, recs_only ? nullptr : out);
    return FQ_OK;
}

int fq_engine_raw_end(fq_engine* e) {
    if (!e) return FQ_E_INVALID;
    if (!e->raw) return FQ_OK;
    for (auto& w : e->raw_queued) e->wait(w->indexed);  // (their host bytes may then be reused)
    e->raw_queued.clear();
    e->raw_prev.reset();
    e->raw = false;
    return FQ_OK;
}

int fq_host_alloc(size_t bytes, void** out) {
    if (!out) return FQ_E_INVALID;
    *out = std::aligned_alloc(4096, (bytes + 4095) / 4096 * 4096);
    return *out ? FQ_OK : FQ_E_NOMEM;
}
int fq_host_free(void* p) {
    std::free(p);
    return FQ_OK;
}
int fq_host_register(const void*, size_t) { return FQ_OK; }
int fq_host_unregister(const void*) { return FQ_OK; }

int fq_dup_create(int, int32_t keylen, fq_dup** out) {
    if (!out) return FQ_E_INVALID;
    *out = new fq_dup{orc_dup_create(keylen)};
    return FQ_OK;
}
int fq_dup_destroy(fq_dup* d) {
    if (!d) return FQ_E_INVALID;
    orc_dup_destroy(d->d);
    delete d;
    return FQ_OK;
}
int fq_engine_set_dup(fq_engine* e, fq_dup* d) {
    if (!e) return FQ_E_INVALID;
    fq_engine_sync(e);
    e->dup = d;
    return FQ_OK;
}
int fq_dup_merge(fq_dup*, const fq_dup*) { return FQ_E_INVALID; }
int fq_dup_stat(fq_dup* d, int32_t hist_size, uint64_t* hist, uint64_t* gc_sum, uint64_t* totals) {
    if (!d) return FQ_E_INVALID;
    orc_dup_stat(d->d, hist_size, hist, gc_sum, totals);
    return FQ_OK;
}

int fq_kmer_open(int device, const uint8_t* seq, const uint32_t* off, int32_t n, fq_kmer_set** out) {
    if (!out) return FQ_E_INVALID;
    if (std::getenv("FQ_CPU_KMER_FAIL")) return FQ_E_NO_DEVICE;  // (tests: the detection fails after the pipeline ran)
    void* k = nullptr;
    const int rc = orc_kmer_open(device, seq, off, n, &k);
    if (rc != FQ_OK) return rc;
    *out = new fq_kmer_set{k};
    return FQ_OK;
}
int fq_kmer_close(fq_kmer_set* s) {
    if (!s) return FQ_E_INVALID;
    orc_kmer_close(s->k);
    delete s;
    return FQ_OK;
}
int fq_kmer_count(fq_kmer_set* s, int32_t keylen, int32_t first, int32_t shift_tail, uint32_t* counts) {
    return s ? orc_kmer_count(s->k, keylen, first, shift_tail, counts) : FQ_E_INVALID;
}
int fq_kmer_find(fq_kmer_set* s, int32_t keylen, int32_t first, int32_t shift_tail, uint32_t seed, uint64_t* occ,
                 size_t cap, size_t* n_out) {
    return s ? orc_kmer_find(s->k, keylen, first, shift_tail, seed, occ, cap, n_out) : FQ_E_INVALID;
}

}  // extern "C"
