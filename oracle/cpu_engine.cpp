// cpu_engine.cpp -- TEST INFRASTRUCTURE ONLY: a CPU stand-in for the host-pack subset of the engine's
// C-ABI (include/fqengine.h), built on the oracle (fq_oracle.c), so the tool's host pipeline
// (fqtool_amd/host: reader, one dispatcher per engine, formatter, writers, pool) can run without a
// GPU under ThreadSanitizer (`make tsan`, tests/test_tsan_cpu.py).  It is linked only into the
// sanitizer build under build/tsan/; the product (fqtool_amd/lib/libfqengine.so) never loads it.
//
// Each engine runs its packs on a worker thread of its own, in submission order, so the host sees
// the same asynchronous contract as the device pipeline: fq_engine_submit returns at once, the host
// batch and `results` are read / written later, fq_engine_poll reports completions in order.
// Text packs and raw streams are GPU-only (they answer FQ_E_INVALID): run the tool with
// FQ_TEXT_MODE=0.  Duplication tables do not merge across engines here (fq_dup_merge fails), so
// -d runs take one engine.
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fq_oracle.h"

struct fq_dup {
    orc_dup* d;
};
struct fq_kmer_set {
    void* k;
};

struct fq_engine {
    fq_params p;
    std::vector<uint64_t> acc;
    fq_dup* dup = nullptr;
    std::string err;
    struct Job {
        fq_batch b;
        fq_read_result* res;
        uint64_t seq;
        int rc;
        bool done;
    };
    std::deque<Job> jobs;  // submitted, in order; front = oldest not yet polled
    std::mutex m;
    std::condition_variable cv;
    bool stop = false;
    std::thread worker;

    void run() {
        std::unique_lock<std::mutex> lk(m);
        for (;;) {
            Job* j = nullptr;
            for (Job& x : jobs)
                if (!x.done) {
                    j = &x;
                    break;
                }
            if (!j) {
                if (stop) return;
                cv.wait(lk);
                continue;
            }
            const fq_batch b = j->b;
            fq_read_result* res = j->res;
            lk.unlock();
            std::vector<uint64_t> a(acc.size(), 0);
            const int rc = orc_process_batch(&p, &b, res, a.data());
            if (rc == FQ_OK && dup) orc_dup_add_batch(dup->d, &b, p.paired);
            lk.lock();
            for (size_t i = 0; i < acc.size(); ++i) acc[i] += a[i];
            j->rc = rc;
            j->done = true;
            cv.notify_all();
        }
    }
};

static int fail(fq_engine* e, int rc, const char* msg) {
    e->err = msg;
    return rc;
}

extern "C" {

int fq_engine_create(const fq_params* params, int device, int32_t max_batch, int32_t max_stride, fq_engine** out) {
    (void)device;
    (void)max_batch;
    (void)max_stride;
    if (!params || !out) return FQ_E_INVALID;
    fq_engine* e = new fq_engine();
    e->p = *params;
    e->acc.assign(fq_acc_words(params->insert_size_max, params->max_cycles), 0);
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
    std::lock_guard<std::mutex> lk(e->m);
    e->jobs.push_back(fq_engine::Job{*b, results, seq_no, 0, false});
    e->cv.notify_all();
    return FQ_OK;
}

int fq_engine_poll(fq_engine* e, int wait, uint64_t* seq_no) {
    if (!e) return FQ_E_INVALID;
    std::unique_lock<std::mutex> lk(e->m);
    if (e->jobs.empty()) return 0;
    if (!e->jobs.front().done) {
        if (!wait) return 0;
        e->cv.wait(lk, [e] { return e->jobs.front().done; });
    }
    const fq_engine::Job j = e->jobs.front();
    e->jobs.pop_front();
    if (seq_no) *seq_no = j.seq;
    if (j.rc != FQ_OK) return fail(e, j.rc, "oracle stand-in: orc_process_batch failed");
    return 1;
}

int fq_engine_pending(const fq_engine* e) {
    if (!e) return FQ_E_INVALID;
    std::lock_guard<std::mutex> lk(const_cast<fq_engine*>(e)->m);
    return (int)e->jobs.size();
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
        for (const auto& j : e->jobs)
            if (!j.done) return false;
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

int fq_engine_submit_text(fq_engine* e, const fq_text_batch*, fq_read_result*, fq_text_out*, uint64_t) {
    return fail(e, FQ_E_INVALID, "oracle stand-in: text packs are GPU-only (FQ_TEXT_MODE=0)");
}
int fq_engine_raw_begin(fq_engine* e, uint64_t, uint64_t) {
    return fail(e, FQ_E_INVALID, "oracle stand-in: raw streams are GPU-only (FQ_TEXT_MODE=0)");
}
int fq_engine_raw_enqueue(fq_engine* e, const fq_raw_window*) { return fail(e, FQ_E_INVALID, "GPU-only"); }
int fq_engine_raw_launch(fq_engine* e, fq_raw_result*, fq_raw_out*, uint64_t) { return fail(e, FQ_E_INVALID, "GPU-only"); }
int fq_engine_raw_end(fq_engine*) { return FQ_OK; }

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
