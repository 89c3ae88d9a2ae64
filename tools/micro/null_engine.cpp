// null_engine.cpp -- PROFILING AID ONLY: an engine library (include/fqengine.h's C-ABI) whose raw
// streams cost nothing, so the fqtool binary's host feed -- the window reader (pread into staging
// windows), the per-engine threads with RawMulti's ordered hand-offs, the formatter hand-off and
// the writers -- runs at its own ceiling with G "infinitely fast" engines (tools/host_feed.py).
//
// Raw windows: the host cuts windows of whole pairs (RawMulti), so a window's pairs are its bytes
// over the fixed record size of the synthetic input (FQ_NULL_REC1 / FQ_NULL_REC2 bytes per record),
// nothing is carried, nothing stops the stream, and every record passes untrimmed: the pack's output
// is as long as its input (the output buffers are not written -- as with the GPU's D2H copies, the
// host pays nothing for them -- so the writers write stale bytes).  Records and accumulators stay
// zero.  Text and host packs complete at once, untouched; only the raw stream is meant to run here.
// Built by tools/host_feed.py into build/nullhost/libfqengine.so, loaded through LD_LIBRARY_PATH.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include <map>
#include <mutex>
#include <sys/mman.h>
#include "../../include/fqengine.h"

struct fq_engine {
    fq_params p;
    size_t acc_words = 0;
    std::string err;
    struct Done {
        uint64_t seq;
        fq_text_out* out;
        uint64_t bytes[2];
    };
    std::deque<Done> pending;
    std::deque<fq_raw_window> queued;
    uint64_t rec[2] = {0, 0};
    uint64_t carry[2] = {0, 0};  // bytes after the last whole record (one engine: windows cut anywhere)
    uint64_t ccap = 0;           // carry capacity (records-only egress: offsets into [carry | window])
    int len = 150;               // read length of the fixed-width records (FQ_NULL_LEN)
    uint64_t max_batch = 0;      // pairs a pack takes at most (as the engine's)
};
struct fq_dup {
    int unused;
};
struct fq_kmer_set {
    int unused;
};

extern "C" {

int fq_engine_create(const fq_params* params, int, int32_t max_batch, int32_t, fq_engine** out) {
    if (!params || !out) return FQ_E_INVALID;
    fq_engine* e = new fq_engine();
    e->max_batch = (uint64_t)max_batch;
    e->p = *params;
    e->acc_words = fq_acc_words(params->insert_size_max, params->max_cycles);
    const char* r1 = std::getenv("FQ_NULL_REC1");
    const char* r2 = std::getenv("FQ_NULL_REC2");
    e->rec[0] = r1 ? std::strtoull(r1, nullptr, 10) : 0;
    e->rec[1] = r2 ? std::strtoull(r2, nullptr, 10) : e->rec[0];
    const char* ln = std::getenv("FQ_NULL_LEN");
    if (ln) e->len = std::atoi(ln);
    *out = e;
    return FQ_OK;
}
int fq_engine_destroy(fq_engine* e) {
    delete e;
    return FQ_OK;
}
size_t fq_engine_acc_words(const fq_engine* e) { return e ? e->acc_words : 0; }
int fq_engine_read_acc(fq_engine* e, uint64_t* host, size_t words) {
    if (!e || !host || words < e->acc_words) return FQ_E_INVALID;
    std::memset(host, 0, e->acc_words * 8);
    return FQ_OK;
}
int fq_engine_reset_acc(fq_engine*) { return FQ_OK; }
int fq_engine_sync(fq_engine*) { return FQ_OK; }
const char* fq_engine_last_error(const fq_engine* e) { return e ? e->err.c_str() : "no engine"; }

int fq_engine_submit(fq_engine* e, const fq_batch*, fq_read_result*, uint64_t seq_no) {
    e->pending.push_back({seq_no, nullptr, {0, 0}});
    return FQ_OK;
}
int fq_engine_submit_text(fq_engine* e, const fq_text_batch* tb, fq_read_result*, fq_text_out* out, uint64_t seq_no) {
    e->pending.push_back({seq_no, out, {tb->text_bytes[0], tb->text_bytes[1]}});
    return FQ_OK;
}
int fq_engine_poll(fq_engine* e, int, uint64_t* seq_no) {
    if (e->pending.empty()) return 0;
    const fq_engine::Done d = e->pending.front();
    e->pending.pop_front();
    if (d.out) {
        d.out->bytes[0] = d.bytes[0];
        d.out->bytes[1] = d.bytes[1];
    }
    if (seq_no) *seq_no = d.seq;
    return 1;
}

int fq_engine_raw_begin(fq_engine* e, uint64_t, uint64_t carry_cap) {
    e->ccap = (carry_cap + 4095) / 4096 * 4096;
    if (!e->rec[0]) {
        e->err = "null engine: set FQ_NULL_REC1 (bytes per record of the fixed-width input)";
        return FQ_E_INVALID;
    }
    e->queued.clear();
    e->carry[0] = e->carry[1] = 0;
    return FQ_OK;
}
int fq_engine_raw_enqueue(fq_engine* e, const fq_raw_window* w) {
    e->queued.push_back(*w);
    return FQ_OK;
}
int fq_engine_raw_launch(fq_engine* e, fq_raw_result* r, fq_raw_out* out, uint64_t seq_no) {
    if (e->queued.empty()) return FQ_E_INVALID;
    const fq_raw_window w = e->queued.front();
    e->queued.pop_front();
    std::memset(r, 0, sizeof *r);
    const int mates = e->p.paired ? 2 : 1;
    uint64_t pairs = ~0ull;
    for (int m = 0; m < mates; ++m) pairs = std::min(pairs, (e->carry[m] + w.n[m]) / e->rec[m]);
    pairs = std::min(pairs, e->max_batch);
    r->pairs = (int32_t)pairs;
    r->max_len = e->len;
    uint64_t cin[2] = {e->carry[0], e->carry[1]};
    for (int m = 0; m < mates; ++m) {
        r->text_bytes[m] = pairs * e->rec[m];
        e->carry[m] = e->carry[m] + w.n[m] - r->text_bytes[m];
        r->carry[m] = e->carry[m];
    }
    out->adapter_bytes[0] = out->adapter_bytes[1] = 0;
    out->text.bytes[0] = out->text.bytes[1] = 0;
    if (out->results) {  // records-only egress: every pair passes, every fourth trimmed by 10 bases
        const int L = e->len;
        for (uint64_t i = 0; i < pairs; ++i)
            for (int m = 0; m < mates; ++m) {
                fq_read_result& rr = out->results[mates * i + m];
                std::memset(&rr, 0, sizeof rr);
                rr.code = FQ_PASS_FILTER;
                rr.len = (uint16_t)(i % 4 == 3 ? L - 10 : L);
                if (i % 4 == 3) {
                    rr.flags = FQ_RF_AD_SEQ;
                    rr.ad_pos = (uint16_t)(L - 10);
                    rr.ad_len = 10;
                }
                fq_text_rec& t = out->rec[m][i];
                t.name_off = (uint32_t)(e->ccap - cin[m] + i * e->rec[m]);
                t.name_len = (uint16_t)(e->rec[m] - 2 * (uint64_t)L - 5);
                t.seq_off = t.name_off + t.name_len + 1;
                t.strand_off = t.seq_off + (uint32_t)L + 1;
                t.strand_len = 1;
                t.qual_off = t.strand_off + 2;
                t.len = (uint16_t)L;
            }
    }
    e->pending.push_back({seq_no, &out->text, {r->text_bytes[0], mates > 1 ? r->text_bytes[1] : 0}});
    return FQ_OK;
}
int fq_engine_raw_wait(fq_engine* e, fq_raw_result* r) {
    if (e->queued.empty()) return FQ_E_INVALID;
    if (r) {  // (the same figures the launch computes, without taking the window)
        std::memset(r, 0, sizeof *r);
        const fq_raw_window& w = e->queued.front();
        const int mates = e->p.paired ? 2 : 1;
        uint64_t pairs = ~0ull;
        for (int m = 0; m < mates; ++m) pairs = std::min(pairs, (e->carry[m] + w.n[m]) / e->rec[m]);
        pairs = std::min(pairs, e->max_batch);
        r->pairs = (int32_t)pairs;
        r->max_len = 150;
        for (int m = 0; m < mates; ++m) {
            r->text_bytes[m] = pairs * e->rec[m];
            r->carry[m] = e->carry[m] + w.n[m] - r->text_bytes[m];
        }
    }
    return FQ_OK;
}
int fq_engine_raw_end(fq_engine* e) {
    e->queued.clear();
    return FQ_OK;
}

// as the engine's (engine.hip): anonymous 2 MiB-page memory populated on the calling thread (the real
// one then registers it with HIP), so the feed's first-touch costs land where the tool's do
static std::mutex g_host_mu;
static std::map<void*, size_t> g_host_maps;
int fq_host_alloc(size_t bytes, void** out) {
    const size_t huge = (size_t)2 << 20;
    const size_t len = ((bytes ? bytes : 1) + huge - 1) / huge * huge;
    void* m = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) return FQ_E_NOMEM;
    (void)madvise(m, len, MADV_HUGEPAGE);
    std::memset(m, 0, len);
    std::lock_guard<std::mutex> g(g_host_mu);
    g_host_maps[m] = len;
    *out = m;
    return FQ_OK;
}
int fq_host_free(void* p) {
    if (!p) return FQ_OK;
    size_t len = 0;
    {
        std::lock_guard<std::mutex> g(g_host_mu);
        auto it = g_host_maps.find(p);
        if (it == g_host_maps.end()) return FQ_E_INVALID;
        len = it->second;
        g_host_maps.erase(it);
    }
    munmap(p, len);
    return FQ_OK;
}

int fq_dup_create(int, int32_t, fq_dup**) { return FQ_E_INVALID; }
int fq_dup_destroy(fq_dup*) { return FQ_OK; }
int fq_dup_merge(fq_dup*, const fq_dup*) { return FQ_E_INVALID; }
int fq_dup_stat(fq_dup*, int32_t, uint64_t*, uint64_t*, uint64_t*) { return FQ_E_INVALID; }
int fq_engine_set_dup(fq_engine*, fq_dup*) { return FQ_OK; }
int fq_kmer_open(int, const uint8_t*, const uint32_t*, int32_t, fq_kmer_set**) { return FQ_E_INVALID; }
int fq_kmer_close(fq_kmer_set*) { return FQ_OK; }
int fq_kmer_count(fq_kmer_set*, int32_t, int32_t, int32_t, uint32_t*) { return FQ_E_INVALID; }
int fq_kmer_find(fq_kmer_set*, int32_t, int32_t, int32_t, uint32_t, uint64_t*, size_t, size_t*) { return FQ_E_INVALID; }

}  // extern "C"
