// processor.cpp -- see processor.h.
#include "processor.h"

#include <algorithm>
#include <atomic>
#include <emmintrin.h>
#include <immintrin.h>
#include <functional>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <iostream>
#include <memory>
#include <mutex>
#include <future>
#include <thread>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "evaluator.h"
#include "pargz.h"

namespace fqhost {
namespace {

// COMMONCONST::FAILED_TYPES, reference src/common.h:21-29
const char* failed_type(int code) {
    switch (code) {
        case 0: return "passed";
        case 4: return "failed_polyx_filter";
        case 8: return "failed_bad_overlap";
        case 12: return "failed_too_many_n_bases";
        case 16: return "failed_too_short";
        case 17: return "failed_too_long";
        case 20: return "failed_quality_filter";
        case 24: return "failed_low_complexity";
        default: return "";
    }
}

char comp(char c) {
    switch (c) {
        case 'A': case 'a': return 'T';
        case 'T': case 't': return 'A';
        case 'C': case 'c': return 'G';
        case 'G': case 'g': return 'C';
        default: return 'N';
    }
}

// A read as the loop body sees it after its in-place edits (fields point into the pack's text).
struct View {
    const char* name;
    size_t name_len;
    const char* strand;
    size_t strand_len;
    const char* seq;
    const char* qual;
    int len;
};

// Read::trimFront of the UMI step (src/read.h:203-208): min(k, len - 1) bases
int umi_cut(int k, int len) { return (k > 0 && len > 0) ? std::min(k, len - 1) : 0; }

// umi_front: the leading bases UmiProcessor::process cut off this mate (Options::umi_front)
View view(const Pack& pk, int m, int i, const fq_read_result* r, int umi_front = 0) {
    const Rec& rc = pk.rec[m][(size_t)i];
    View v{pk.name(m, (size_t)i), rc.name_len, pk.strand(m, (size_t)i), rc.strand_len,
           pk.seq_text(m, (size_t)i), pk.qual_text(m, (size_t)i), (int)rc.len};
    if (r && !(r->flags & FQ_RF_NULL)) {  // trimmed in place
        v.seq += r->start;
        v.qual += r->start;
        v.len = r->len;
    } else if (umi_front) {  // a NULL read keeps the (UMI-trimmed) original
        const int u = umi_cut(umi_front, v.len);
        v.seq += u;
        v.qual += u;
        v.len -= u;
    }
    return v;
}

// Read::firstIndex, reference src/read.h:107-124 (sic: with two indexes the character before
// the '+' is dropped)
std::string first_index(const char* name, size_t n) {
    const int len = (int)n;
    int end = len;
    if (len < 5) return "";
    for (int i = len - 3; i >= 0; --i) {
        if (name[i] == '+') end = i - 1;
        if (name[i] == ':') return std::string(name, n).substr((size_t)i + 1, (size_t)(end - i));
    }
    return "";
}

// UmiProcessor::process (src/umiprocessor.cpp:10-79): the tag appended to both names, or ""
std::string umi_tag(const Options& o, const Pack& pk, int i) {
    std::string umi = " OX:Z:", qua = " BZ:Z:";
    const int L = o.umi_length;
    const bool pe = pk.paired;
    const int len1 = (int)pk.rec[0][(size_t)i].len, len2 = pe ? (int)pk.rec[1][(size_t)i].len : 0;
    auto idx = [&](int m) { return first_index(pk.name(m, (size_t)i), pk.rec[m][(size_t)i].name_len); };
    // the original text (UMI runs before base correction, src/peprocessor.cpp:288-312)
    auto seq = [&](int m, int from, int n) {
        return std::string(pk.arena(m) + pk.rec[m][(size_t)i].seq_off() + from, (size_t)n);
    };
    auto qual = [&](int m, int from, int n) {
        return std::string(pk.arena(m) + pk.rec[m][(size_t)i].qual_off() + from, (size_t)n);
    };
    const int cut1 = o.umi_not_trim ? 0 : umi_cut(L + o.umi_skip, len1);
    const int cut2 = o.umi_not_trim ? 0 : umi_cut(L + o.umi_skip, len2);
    switch (o.umi_location) {
        case 1: umi += idx(0); break;
        case 2:
            if (pe) umi += idx(1);
            break;
        case 3:
            umi += seq(0, 0, std::min(len1, L));
            qua += qual(0, 0, std::min(len1, L));
            break;
        case 4:
            if (pe) {
                umi += seq(1, 0, std::min(len2, L));
                qua += qual(1, 0, std::min(std::min(len1, L), len2));  // sic: r1's length (:44)
            }
            break;
        case 5:
            umi += idx(0);
            if (pe) umi += "-" + idx(1);
            break;
        case 6:
            umi += seq(0, 0, std::min(len1, L));
            qua += qual(0, 0, std::min(len1, L));
            if (pe) {  // r2's quality is taken after its trim, bounded by r1's trimmed length (:64-67)
                umi += "-" + seq(1, 0, std::min(len2, L));
                qua += "-" + qual(1, cut2, std::min(std::min(len1 - cut1, L), len2 - cut2));
            }
            break;
        default: break;
    }
    std::string tag = umi;
    if (tag.size() > 6 && qua.size() > 6) tag += qua;
    return tag.size() > 6 ? tag : std::string();
}

// UmiProcessor::addTagToName, src/umiprocessor.cpp:81-89
std::string tagged_name(const char* name, size_t n, const std::string& tag, bool drop_comment) {
    const std::string s(name, n);
    const size_t pos = s.find_first_of(' ');
    if (pos == std::string::npos) return s + tag;
    if (drop_comment) return s.substr(0, pos) + tag;
    return s.substr(0, pos) + tag + s.substr(pos);
}

// Read::toString / toStringWithTag, reference src/read.h:166-178
void append_read(std::string& out, const View& v, const char* tag = nullptr) {
    out.append(v.name, v.name_len);
    if (tag) {
        out += ' ';
        out += tag;
    }
    out += '\n';
    out.append(v.seq, (size_t)v.len);
    out += '\n';
    out.append(v.strand, v.strand_len);
    out += '\n';
    out.append(v.qual, (size_t)v.len);
    out += '\n';
}

// text bytes of mate m's records [i0, i1) plus their line breaks: their untrimmed output size
size_t span_bytes(const Pack& pk, int m, int i0, int i1) {
    if (i1 <= i0) return 0;
    const Rec& a = pk.rec[m][(size_t)i0];
    const Rec& b = pk.rec[m][(size_t)i1 - 1];
    return (size_t)(b.off - a.off) + b.name_len + 2 * (size_t)b.len + b.strand_len + 4 * (size_t)(i1 - i0);
}

// the loop bodies' appends for reads (pairs) [i0, i1), into block k of each destination
void format_range(const Options& o, const Pack& pk, const fq_read_result* res, int i0, int i1, size_t k,
                  PackOutput& out) {
    const bool has_unpaired_left = !o.unpaired1.empty();
    const bool has_failed = !o.failed_out.empty();
    std::string& o1 = out.out1[k];
    std::string& o2 = out.out2[k];
    std::string& u1 = out.unpaired1[k];
    std::string& u2 = out.unpaired2[k];
    std::string& fl = out.failed[k];
    std::string& mg = out.merged[k];
    const int uf1 = o.umi_front(0), uf2 = o.umi_front(1);
    std::string name1, name2;  // UMI-tagged names
    auto apply_umi = [&](int i, View& v1, View* v2) {
        const std::string tag = umi_tag(o, pk, i);
        if (tag.empty()) return;
        name1 = tagged_name(v1.name, v1.name_len, tag, o.umi_drop_comment);
        v1.name = name1.data();
        v1.name_len = name1.size();
        if (v2) {
            name2 = tagged_name(v2->name, v2->name_len, tag, o.umi_drop_comment);
            v2->name = name2.data();
            v2->name_len = name2.size();
        }
    };
    if (!pk.paired) {  // src/seprocessor.cpp:337-350
        for (int i = i0; i < i1; ++i) {
            const fq_read_result& r = res[i];
            if (r.flags & FQ_RF_INDEX_FILTERED) continue;  // :304-307
            View v = view(pk, 0, i, &r, uf1);
            if (o.umi) apply_umi(i, v, nullptr);
            if (!(r.flags & FQ_RF_NULL) && r.code == FQ_PASS_FILTER) append_read(o1, v);
            else if (has_failed) append_read(fl, v, failed_type(r.code));
        }
        return;
    }
    for (int i = i0; i < i1; ++i) {  // src/peprocessor.cpp:351-429
        const fq_read_result& a = res[2 * (size_t)i];
        const fq_read_result& b = res[2 * (size_t)i + 1];
        if (a.flags & FQ_RF_INDEX_FILTERED) continue;  // :283-286
        const bool nn1 = !(a.flags & FQ_RF_NULL), nn2 = !(b.flags & FQ_RF_NULL);
        View v1 = view(pk, 0, i, &a, uf1), v2 = view(pk, 1, i, &b, uf2);
        if (o.umi) apply_umi(i, v1, &v2);
        bool merge_processed = false;
        if (o.merge && nn1 && nn2) {
            if (a.flags & FQ_RF_MERGED) {
                if (a.code == FQ_PASS_FILTER) {  // OverlapAnalysis::merge, src/overlapanalysis.cpp:74-104
                    const int m1 = a.m_len1, m2 = a.m_len2, ol = v2.len - m2;
                    std::string seq(v1.seq, (size_t)m1), qual(v1.qual, (size_t)m1);
                    for (int j = 0; j < m2; ++j) {
                        const int src = v2.len - 1 - (ol + j);
                        seq += comp(v2.seq[src]);
                        qual += v2.qual[src];
                    }
                    const std::string name = merged_name(std::string(v1.name, v1.name_len), m1, m2);
                    const View mv{name.data(), name.size(), v1.strand, v1.strand_len, seq.data(), qual.data(),
                                  (int)seq.size()};
                    append_read(mg, mv);
                }
                merge_processed = true;
            } else if (!o.discard_unmerged) {
                if (a.code == FQ_PASS_FILTER) append_read(mg, v1);
                if (b.code == FQ_PASS_FILTER) append_read(mg, v2);
                merge_processed = true;
            }
        }
        if (merge_processed) continue;
        const bool p1 = nn1 && a.code == FQ_PASS_FILTER, p2 = nn2 && b.code == FQ_PASS_FILTER;
        if (p1 && p2) {
            append_read(o1, v1);
            append_read(o2, v2);
        } else if (p1) {
            if (has_unpaired_left) {
                append_read(u1, v1);
                if (has_failed) append_read(fl, v2, failed_type(b.code));
            } else if (has_failed) {
                append_read(fl, v1, "paired_read_is_failing");
                append_read(fl, v2, failed_type(b.code));
            }
        } else if (p2) {
            if (has_unpaired_left) {  // the reference checks the LEFT writer here (src/peprocessor.cpp:417)
                append_read(u2, v2);
                if (has_failed) append_read(fl, v1, failed_type(b.code));  // sic: result2 (:420)
            } else if (has_failed) {
                append_read(fl, v1, failed_type(a.code));
                append_read(fl, v2, "paired_read_is_failing");
            }
        }
    }
}

}  // namespace

std::string merged_name(const std::string& name, int len1, int len2) {
    const std::string tag = "_merged_" + std::to_string(len1) + "_" + std::to_string(len2);
    const size_t pos = name.find_first_of(' ');
    if (pos == std::string::npos) return tag;
    return name.substr(0, pos - 1) + tag + name.substr(pos);
}

// Filter::match, reference src/filter.cpp:191-207
bool index_match(const std::vector<std::string>& list, const std::string& target, int threshold) {
    const size_t tlen = target.size();
    for (const std::string& s : list) {
        int diff = 0;
        for (size_t k = 0; k < s.size() && k < tlen; ++k)
            if (s[k] != target[k] && ++diff > threshold) break;
        if (diff <= threshold) return true;
    }
    return false;
}

void prepare_pack(const Options& o, Pack& pk, Pool* pool) {
    pk.use_flags = o.index_filter;
    if (!o.index_filter) return;
    pk.flags.resize((size_t)pk.n);
    const int parts = pool ? std::max(1, std::min(pool->size() * 2, (pk.n + 16383) / 16384)) : 1;
    auto work = [&](int k) {
        const int i0 = (int)((int64_t)pk.n * k / parts), i1 = (int)((int64_t)pk.n * (k + 1) / parts);
        for (int i = i0; i < i1; ++i) {  // Filter::filterByIndex, src/filter.cpp:209-232
            bool hit = index_match(o.blacklist1, first_index(pk.name(0, (size_t)i), pk.rec[0][(size_t)i].name_len),
                                   o.index_threshold);
            if (!hit && pk.paired)
                hit = index_match(o.blacklist2, first_index(pk.name(1, (size_t)i), pk.rec[1][(size_t)i].name_len),
                                  o.index_threshold);
            pk.flags[(size_t)i] = hit ? FQ_BF_INDEX_FILTERED : 0;
        }
    };
    if (pool) pool->run(parts, work);
    else work(0);
}

void apply_corrections(const Options& o, Pack& pk, const fq_read_result* res, Pool* pool) {
    pk.fix.clear();
    pk.fix_arena.clear();
    if (!o.correction || !pk.paired) return;
    const int parts = pool ? std::max(1, std::min(pool->size() * 2, (pk.n + 16383) / 16384)) : 1;
    pk.fix.assign((size_t)pk.n, nullptr);
    pk.fix_arena.resize((size_t)parts);
    auto work = [&](int k) {
        const int i0 = (int)((int64_t)pk.n * k / parts), i1 = (int)((int64_t)pk.n * (k + 1) / parts);
        auto corrected = [&](int i) { return ((res[2 * (size_t)i].flags | res[2 * (size_t)i + 1].flags) & FQ_RF_CORRECTED) != 0; };
        size_t bytes = 0;
        for (int i = i0; i < i1; ++i)
            if (corrected(i)) bytes += 2 * ((size_t)pk.rec[0][(size_t)i].len + pk.rec[1][(size_t)i].len);
        std::string& ar = pk.fix_arena[(size_t)k];
        ar.resize(bytes);
        size_t at = 0;
        for (int i = i0; i < i1; ++i) {
            if (!corrected(i)) continue;
            const size_t l1 = pk.rec[0][(size_t)i].len, l2 = pk.rec[1][(size_t)i].len;
            char* d = &ar[at];
            std::memcpy(d, pk.seq_text(0, (size_t)i), l1);
            std::memcpy(d + l1, pk.qual_text(0, (size_t)i), l1);
            std::memcpy(d + 2 * l1, pk.seq_text(1, (size_t)i), l2);
            std::memcpy(d + 2 * l1 + l2, pk.qual_text(1, (size_t)i), l2);
            const fq_read_result& a = res[2 * (size_t)i];
            const fq_read_result& b = res[2 * (size_t)i + 1];
            fq_correct_pair_text(d + a.start, d + l1 + a.start, d + 2 * l1 + b.start, d + 2 * l1 + l2 + b.start,
                                 (int16_t)b.m_len1, b.m_len2, b.reserved);
            pk.fix[(size_t)i] = d;
            at += 2 * (l1 + l2);
        }
    };
    if (pool) pool->run(parts, work);
    else work(0);
}

void format_pack(const Options& o, const Pack& pk, const fq_read_result* res, PackOutput& out, Pool* pool,
                 const std::vector<int>* cuts) {
    const int parts = cuts ? std::max(0, (int)cuts->size() - 1)
                           : pool ? std::max(1, std::min(pool->size() * 2, (pk.n + 8191) / 8192)) : 1;
    for (auto* v : {&out.out1, &out.out2, &out.unpaired1, &out.unpaired2, &out.failed, &out.merged}) {
        v->clear();
        v->resize((size_t)parts);
    }
    auto work = [&](int k) {
        const int i0 = cuts ? (*cuts)[(size_t)k] : (int)((int64_t)pk.n * k / parts);
        const int i1 = cuts ? (*cuts)[(size_t)k + 1] : (int)((int64_t)pk.n * (k + 1) / parts);
        out.out1[(size_t)k].reserve(span_bytes(pk, 0, i0, i1));
        if (pk.paired) {
            if (o.merge) out.merged[(size_t)k].reserve(span_bytes(pk, 0, i0, i1) + span_bytes(pk, 1, i0, i1));
            else out.out2[(size_t)k].reserve(span_bytes(pk, 1, i0, i1));
        }
        format_range(o, pk, res, i0, i1, (size_t)k, out);
    };
    if (pool && parts > 1) pool->run(parts, work);
    else
        for (int k = 0; k < parts; ++k) work(k);
}

namespace {

template <class T>
class Queue {  // bounded FIFO between pipeline threads; push/pop return at once after close()
   public:
    explicit Queue(size_t cap) : cap_(cap) {}
    bool push(T v) {  // false: the queue was closed and v dropped
        std::unique_lock<std::mutex> l(m_);
        not_full_.wait(l, [&] { return q_.size() < cap_ || closed_; });
        if (closed_) return false;
        q_.push_back(std::move(v));
        not_empty_.notify_one();
        return true;
    }
    bool pop(T& v) {
        std::unique_lock<std::mutex> l(m_);
        not_empty_.wait(l, [&] { return !q_.empty() || closed_; });
        if (q_.empty()) return false;
        v = std::move(q_.front());
        q_.pop_front();
        not_full_.notify_one();
        return true;
    }
    // pop of the most recently pushed element (a stack of recycled buffers: the warm ones go out
    // again first, the cold ones stay untouched -- never page-locked -- unless demand needs them)
    bool pop_recent(T& v) {
        std::unique_lock<std::mutex> l(m_);
        not_empty_.wait(l, [&] { return !q_.empty() || closed_; });
        if (q_.empty()) return false;
        v = std::move(q_.back());
        q_.pop_back();
        not_full_.notify_one();
        return true;
    }
    // pop / pop_recent waiting at most d: 1 taken, 0 timed out, -1 closed and drained
    int pop_for(T& v, std::chrono::microseconds d, bool recent = false) {
        std::unique_lock<std::mutex> l(m_);
        // (system_clock: see Lane::run_raw_multi's wait_polling)
        if (!not_empty_.wait_until(l, std::chrono::system_clock::now() + d, [&] { return !q_.empty() || closed_; })) return 0;
        if (q_.empty()) return -1;
        if (recent) {
            v = std::move(q_.back());
            q_.pop_back();
        } else {
            v = std::move(q_.front());
            q_.pop_front();
        }
        not_full_.notify_one();
        return 1;
    }
    // pop_recent without waiting: 1 taken, 0 empty (not closed), -1 closed and drained
    int try_pop_recent(T& v) {
        std::lock_guard<std::mutex> l(m_);
        if (q_.empty()) return closed_ ? -1 : 0;
        v = std::move(q_.back());
        q_.pop_back();
        not_full_.notify_one();
        return 1;
    }
    // 1: v taken; 0: empty (not closed); -1: closed and drained
    int try_pop(T& v) {
        std::lock_guard<std::mutex> l(m_);
        if (q_.empty()) return closed_ ? -1 : 0;
        v = std::move(q_.front());
        q_.pop_front();
        not_full_.notify_one();
        return 1;
    }
    void close() {
        std::lock_guard<std::mutex> l(m_);
        closed_ = true;
        not_empty_.notify_all();
        not_full_.notify_all();
    }
    void reopen() {
        std::lock_guard<std::mutex> l(m_);
        closed_ = false;
    }

   private:
    size_t cap_;
    std::deque<T> q_;
    bool closed_ = false;
    std::mutex m_;
    std::condition_variable not_full_, not_empty_;
};

}  // namespace

// WriterThread (src/writerthread.cpp): one thread per output file, blocks written in order.
// A write error (full disk, deflate failure) stops the thread and is rethrown by close().
// A plain regular file takes its raw texts (packs) on kIoThreads threads at once: the writer
// thread claims each text's byte range in output order and an I/O thread pwrites it there (one
// thread's copies into the page cache ran at ~4 GB/s; bench e2e_file).
class AsyncWriter {
   public:
    static constexpr int kIoThreads = 4;
    AsyncWriter(const std::string& path, int level, Pool* pool) : w_(path, level), pool_(pool), q_(4) {
        if (w_.positional()) {
            io_.reset(new Queue<Io>(kIoThreads));
            for (int i = 0; i < kIoThreads; ++i) io_t_.emplace_back([this] { io_loop(); });
        }
        t_ = std::thread([this] { loop(); });
    }
    ~AsyncWriter() {
        try {
            close();
        } catch (...) {
        }
    }
    void write(std::vector<std::string> blocks) {
        if (failed_) std::rethrow_exception(error());
        bool any = false;
        for (const auto& s : blocks) any = any || !s.empty();
        if (any && !q_.push(Job{std::move(blocks), nullptr, 0, nullptr, nullptr}) && failed_) std::rethrow_exception(error());
    }
    // queue n bytes at p (which stay valid until `done` runs); the writer thread runs it once the
    // bytes are written (or dropped after a write error)
    void write_raw(const char* p, size_t n, std::function<void()> done) {
        if (failed_ || !q_.push(Job{{}, p, n, done, nullptr})) {
            done();  // (the writer has stopped: nothing will take the text)
            if (failed_) std::rethrow_exception(error());
            throw std::runtime_error("write to a closed output");
        }
    }
    // queue byte ranges (plain outputs; they stay valid until `done` runs), as write_raw
    void write_segs(const std::vector<iovec>* segs, std::function<void()> done) {
        if (failed_ || !q_.push(Job{{}, nullptr, 0, done, segs})) {
            done();
            if (failed_) std::rethrow_exception(error());
            throw std::runtime_error("write to a closed output");
        }
    }
    bool gzip() const { return w_.gzip(); }
    void close() {
        if (closed_) return;
        closed_ = true;
        q_.close();
        t_.join();
        if (io_) {  // (the ranges claimed so far are written, or failed)
            io_->close();
            for (auto& t : io_t_) t.join();
        }
        if (!failed_) {
            try {
                w_.close();
            } catch (...) {
                fail(std::current_exception());
            }
        }
        if (failed_) std::rethrow_exception(error());
    }

   private:
    struct Job {
        std::vector<std::string> blocks;
        const char* raw;
        size_t raw_n;
        std::function<void()> done;
        const std::vector<iovec>* segs = nullptr;
    };
    struct Io {
        uint64_t off;
        Job job;
    };
    void io_loop() {
        Io x;
        while (io_->pop(x)) {
            try {
                if (!failed_) {  // (after a failure the claimed ranges are dropped)
                    if (x.job.segs) w_.write_segs_at(x.off, x.job.segs->data(), x.job.segs->size());
                    else w_.write_at(x.off, x.job.raw, x.job.raw_n);
                }
            } catch (...) {
                // (e.g. ENOSPC) visible to the producers at once: their next write rethrows it, the
                // writer thread stops claiming ranges and releases what is queued
                fail(std::current_exception());
                q_.close();
            }
            x.job.done();
        }
    }
    void loop() {
        Job j;
        try {
            while (q_.pop(j)) {
                if (failed_) {  // (an I/O thread's write failed: this job is released, the rest below)
                    if (j.done) j.done();
                    std::rethrow_exception(error());
                }
                if (j.done && io_) {  // claim the range here (output order), write it on an I/O thread
                    size_t n = j.raw_n;
                    if (j.segs) {
                        n = 0;
                        for (const iovec& v : *j.segs) n += v.iov_len;
                    }
                    const uint64_t off = w_.claim(n);
                    std::function<void()> done = j.done;
                    if (!io_->push(Io{off, std::move(j)})) done();
                    j = Job{};
                } else if (j.done) {
                    try {
                        if (j.segs) w_.write_segs(j.segs->data(), j.segs->size());
                        else w_.write_raw(j.raw, j.raw_n, pool_);
                    } catch (...) {
                        j.done();
                        throw;
                    }
                    j.done();
                } else {
                    w_.write(j.blocks, pool_);
                }
            }
        } catch (...) {
            fail(std::current_exception());
            q_.close();  // the producer's next push returns at once; write() rethrows
            while (q_.pop(j))  // (raw jobs queued behind the failure are released)
                if (j.done) j.done();
        }
    }
    // the first error of the writer or an I/O thread; producers see failed_ without the lock
    void fail(std::exception_ptr e) {
        std::lock_guard<std::mutex> g(err_m_);
        if (!err_) err_ = e;
        failed_ = true;
    }
    std::exception_ptr error() {
        std::lock_guard<std::mutex> g(err_m_);
        return err_;
    }
    Writer w_;
    Pool* pool_;
    Queue<Job> q_;
    std::mutex err_m_;
    std::exception_ptr err_;
    std::atomic<bool> failed_{false};
    bool closed_ = false;
    std::unique_ptr<Queue<Io>> io_;
    std::vector<std::thread> io_t_;
    std::thread t_;
};

OutputSet::OutputSet(const Options& o, Pool* pool) : paired_(o.paired()) {
    const int z = o.compression;
    if (paired_) {
        if (!o.unpaired1.empty()) wu1_.reset(new AsyncWriter(o.unpaired1, z, pool));
        if (!o.unpaired2.empty() && o.unpaired2 != o.unpaired1) wu2_.reset(new AsyncWriter(o.unpaired2, z, pool));
        if (o.merge && !o.merge_out.empty()) wm_.reset(new AsyncWriter(o.merge_out, z, pool));
    }
    if (!o.failed_out.empty()) wf_.reset(new AsyncWriter(o.failed_out, z, pool));
    if (!o.out1.empty()) {
        w1_.reset(new AsyncWriter(o.out1, z, pool));
        if (paired_ && !o.out2.empty()) w2_.reset(new AsyncWriter(o.out2, z, pool));
    }
}

OutputSet::~OutputSet() {
    try {
        close();
    } catch (...) {
    }
}

void OutputSet::write(PackOutput&& out) {
    if (wm_) wm_->write(std::move(out.merged));
    if (wf_) wf_->write(std::move(out.failed));
    if (w1_ && (!paired_ || w2_)) {  // PE writes the pair outputs only with both writers (:469)
        w1_->write(std::move(out.out1));
        if (w2_) w2_->write(std::move(out.out2));
    }
    if (wu1_) wu1_->write(std::move(out.unpaired1));
    if (wu2_) wu2_->write(std::move(out.unpaired2));
}

void OutputSet::write_text(const char* t1, size_t n1, const char* t2, size_t n2, std::function<void()> done) {
    if (!(w1_ && (!paired_ || w2_))) {  // PE writes the pair outputs only with both writers (:469)
        done();
        return;
    }
    // `done` runs once, when the last writer is through with its text
    auto left = std::make_shared<std::atomic<int>>(w2_ ? 2 : 1);
    auto fin = [left, done] {
        if (left->fetch_sub(1) == 1) done();
    };
    std::exception_ptr err;
    try {
        w1_->write_raw(t1, n1, fin);
    } catch (...) {
        err = std::current_exception();
    }
    if (w2_) {
        try {
            w2_->write_raw(t2, n2, fin);
        } catch (...) {
            if (!err) err = std::current_exception();
        }
    }
    if (err) std::rethrow_exception(err);
}

void OutputSet::write_text_segs(const std::vector<iovec>& s1, const std::vector<iovec>& s2, std::function<void()> done) {
    if (!(w1_ && (!paired_ || w2_))) {
        done();
        return;
    }
    auto left = std::make_shared<std::atomic<int>>(w2_ ? 2 : 1);
    auto fin = [left, done] {
        if (left->fetch_sub(1) == 1) done();
    };
    std::exception_ptr err;
    try {
        w1_->write_segs(&s1, fin);
    } catch (...) {
        err = std::current_exception();
    }
    if (w2_) {
        try {
            w2_->write_segs(&s2, fin);
        } catch (...) {
            if (!err) err = std::current_exception();
        }
    }
    if (err) std::rethrow_exception(err);
}

bool OutputSet::plain_pair_outputs() const { return (!w1_ || !w1_->gzip()) && (!w2_ || !w2_->gzip()); }

void OutputSet::write_merged_text(const char* t, size_t n, std::function<void()> done) {
    if (!wm_) {
        done();
        return;
    }
    wm_->write_raw(t, n, std::move(done));
}

void OutputSet::close() {
    std::exception_ptr first;
    for (auto* w : {&w1_, &w2_, &wu1_, &wu2_, &wf_, &wm_}) {
        if (!*w) continue;
        try {
            (*w)->close();
        } catch (...) {
            if (!first) first = std::current_exception();
        }
        w->reset();
    }
    if (first) std::rethrow_exception(first);
}

namespace {

// util::replace / basename / dirname / joinpath, reference src/util.h:121-250
std::string home_path(const std::string& path) {
    const char* h = std::getenv("HOME");
    const std::string des = std::string(h ? h : "") + "/";
    std::string ret;
    size_t las = 0, cur = 0;
    while ((cur = path.find('~', cur)) != std::string::npos) {
        ret.append(path.substr(las, cur - las)).append(des);
        las = ++cur;
    }
    return ret + path.substr(las);
}

std::string path_basename(const std::string& path) {
    const std::string f = home_path(path);
    if (f.find_first_of(" \t\n\v\f\r") != std::string::npos) return "";
    const size_t p1 = f.find_last_of("/\\");
    if (p1 == std::string::npos) return f;
    const size_t p2 = f.find_last_not_of("/\\");
    if (p2 == f.size() - 1) return f.substr(p1 + 1, p2 - p1);
    const size_t p3 = f.find_last_of("/\\", p2);
    if (p3 == std::string::npos) return f.substr(0, p2 + 1);
    return f.substr(p3 + 1, p2 - p3);
}

std::string path_dirname(const std::string& path) {
    const std::string f = home_path(path);
    const size_t pos = f.find_last_of("/\\");
    if (pos == std::string::npos) return "./";
    if (pos == f.size() - 1) {
        const size_t p1 = f.find_last_not_of("/\\");
        if (p1 == std::string::npos) return "/";
        const size_t p2 = f.find_last_of("/\\", p1);
        return p2 == std::string::npos ? "./" : f.substr(0, p2 + 1);
    }
    return f.substr(0, pos + 1);
}

}  // namespace

// The split outputs of -s / -S: ThreadConfig::initWriterForSplit / markProcessed /
// writeEmptyFilesForSplitting (src/threadconfig.cpp:88-137) with the reference's packs of
// --max_item_in_pack pairs.  Worker t of -w T writes files t+1, t+1+T, ... (4-digit prefix,
// src/options.h:272); a pack's passing pairs go to its worker's current file, then the worker
// moves on once it has seen split_size pairs (-s: packed pairs; -S: passed pairs).  With -w 1
// (the reference's deterministic setting) this is the reference's output; with more workers the
// packs are dealt round-robin over the workers still running, one schedule the reference can take.
// Unpaired / failed / merged outputs are not written in split mode (PairEndProcessor::process
// skips initOutput).
class SplitSink {
   public:
    SplitSink(const Options& o, Pool* pool) : o_(o), pool_(pool), T_(std::max(1, o.threads)), th_((size_t)T_) {
        for (int t = 0; t < T_; ++t) {
            th_[(size_t)t].working = t;
            open(t);
        }
    }
    void write(const Pack& pk, const fq_read_result* res, uint64_t first) {
        const uint64_t P = std::max<uint64_t>(1, o_.max_reads_in_pack);
        std::vector<int> cuts{0};
        for (int i = 0; i < pk.n;) {  // blocks never straddle a reference pack
            const uint64_t g = first + (uint64_t)i;
            const int end = (int)std::min<uint64_t>((uint64_t)pk.n, (g / P + 1) * P - first);
            const int step = std::min(end - i, 16384);
            i += step;
            cuts.push_back(i);
        }
        PackOutput out;
        format_pack(o_, pk, res, out, pool_, &cuts);
        for (size_t j = 0; j + 1 < cuts.size(); ++j) {
            const uint64_t ref = (first + (uint64_t)cuts[j]) / P;
            if (!have_ref_ || ref != ref_) {
                finish_ref();
                start_ref(ref);
            }
            Worker& w = th_[(size_t)t_];
            if (w.w1) w.w1->write(std::vector<std::string>{std::move(out.out1[j])}, pool_);
            if (w.w2) w.w2->write(std::vector<std::string>{std::move(out.out2[j])}, pool_);
            count_ += (uint64_t)(cuts[j + 1] - cuts[j]);
            passed_ += passed(pk, res, cuts[j], cuts[j + 1]);
        }
    }
    void close() {
        finish_ref();
        for (int t = 0; t < T_; ++t) {
            Worker& w = th_[(size_t)t];
            if (o_.split_by_number)  // writeEmptyFilesForSplitting
                while (w.working + T_ < o_.split_number) {
                    w.working += T_;
                    open(t);
                }
            if (w.w1) w.w1->close();
            if (w.w2) w.w2->close();
            w.w1.reset();
            w.w2.reset();
        }
    }

   private:
    struct Worker {
        int working = 0;
        uint64_t cur = 0;
        bool stopped = false;
        std::unique_ptr<Writer> w1, w2;
    };
    // readPassed of the loop bodies (src/peprocessor.cpp:380-403, src/seprocessor.cpp:341-345)
    uint64_t passed(const Pack& pk, const fq_read_result* res, int i0, int i1) const {
        uint64_t n = 0;
        auto ok = [](const fq_read_result& r) { return !(r.flags & (FQ_RF_NULL | FQ_RF_INDEX_FILTERED)) && r.code == FQ_PASS_FILTER; };
        for (int i = i0; i < i1; ++i)
            n += pk.paired ? (ok(res[2 * (size_t)i]) && ok(res[2 * (size_t)i + 1])) : ok(res[i]);
        return n;
    }
    void open(int t) {  // initWriterForSplit
        Worker& w = th_[(size_t)t];
        if (w.w1) w.w1->close();
        if (w.w2) w.w2->close();
        w.w1.reset();
        w.w2.reset();
        std::string num = std::to_string(w.working + 1);
        while (num.size() < 4) num = "0" + num;
        w.w1.reset(new Writer(path_dirname(o_.out1) + "/" + num + "." + path_basename(o_.out1), o_.compression));
        if (o_.paired())
            w.w2.reset(new Writer(path_dirname(o_.out2) + "/" + num + "." + path_basename(o_.out2), o_.compression));
    }
    void start_ref(uint64_t ref) {
        for (int k = 0; k < T_; ++k) {  // the next worker still taking packs
            const int t = (next_ + k) % T_;
            if (!th_[(size_t)t].stopped) {
                t_ = t;
                next_ = (t + 1) % T_;
                break;
            }
        }
        ref_ = ref;
        have_ref_ = true;
        count_ = passed_ = 0;
    }
    void finish_ref() {  // markProcessed
        if (!have_ref_) return;
        have_ref_ = false;
        Worker& w = th_[(size_t)t_];
        w.cur += o_.split_by_lines ? passed_ : count_;
        if (w.cur >= o_.split_size) {
            if (o_.split_by_lines || w.working + T_ < o_.split_number) {
                w.working += T_;
                open(t_);
                w.cur = 0;
            } else if (o_.split_number % T_ > 0 && t_ >= o_.split_number % T_) {
                w.stopped = true;
            }
        }
    }
    const Options& o_;
    Pool* pool_;
    int T_;
    std::vector<Worker> th_;
    int t_ = 0, next_ = 0;
    uint64_t ref_ = 0, count_ = 0, passed_ = 0;
    bool have_ref_ = false;
};

Sink::Sink(const Options& o, Pool* pool) : o_(o), pool_(pool), merge_(o.merge && o.paired()) {
    if (o.split()) split_.reset(new SplitSink(o, pool));
    else outs_.reset(new OutputSet(o, pool));
}

Sink::~Sink() {
    try {
        close();
    } catch (...) {
    }
}

void Sink::consume(const Pack& pk, const fq_read_result* res) {
    if (split_) {
        split_->write(pk, res, pairs_);
    } else {
        PackOutput out;
        format_pack(o_, pk, res, out, pool_);
        outs_->write(std::move(out));
    }
    pairs_ += (uint64_t)pk.n;
}

bool Sink::plain_pair_outputs() const { return outs_ && !merge_ && outs_->plain_pair_outputs(); }

void Sink::consume_text(const Pack& pk, std::function<void()> done) {
    pairs_ += (uint64_t)pk.n;
    if (pk.zc) outs_->write_text_segs(pk.segs[0], pk.segs[1], std::move(done));
    else if (merge_) outs_->write_merged_text(pk.out_text[0].data(), pk.tout.bytes[0], std::move(done));
    else outs_->write_text(pk.out_text[0].data(), pk.tout.bytes[0], pk.out_text[1].data(), pk.tout.bytes[1], std::move(done));
}

void Sink::close() {
    if (split_) split_->close();
    if (outs_) outs_->close();
    split_.reset();
    outs_.reset();
}

namespace {

int round16(int x) { return (x + 15) & ~15; }

bool ends_with_gz(const std::string& f) { return f.size() >= 3 && f.compare(f.size() - 3, 3, ".gz") == 0; }

double since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
}

struct Stopped {};  // another pipeline stage failed and closed the queues

// Records-only raw packs (fq_raw_out.results): the output text and the trimmed-adapter entries built
// on the host from its staging window, as text.hip's text_write_kernel and raw.hip's entries do on
// the device (Read::toString of the passing records in input order, src/read.h:166-168,
// src/peprocessor.cpp:457-491; FilterResult::addAdapterTrimmed's strings).  The window's carry (the
// previous pack's unconsumed bytes) is copied in front of it first, from the previous pack's
// window, which is then returned to the window reader.
struct RawPrev {
    char* buf[2] = {nullptr, nullptr};
    uint64_t end[2] = {0, 0};
    std::shared_ptr<void> hold;  // the previous pack's window, until the next carry is copied from it
};

// zc (zero copy, plain outputs): the output is byte ranges (Pack::segs) -- runs of records that pass
// untrimmed stay in the staging window, only trimmed records are formatted (into out_text) -- and
// the pack holds its window until the writers are through with it.
void format_raw_recs(Pack& pk, RawPrev& prev, bool adapters, const fq_params& p, Pool& pool, AdapterCounts& ac, bool zc) {
    const int mates = pk.paired ? 2 : 1;
    for (int m = 0; m < mates; ++m) {
        char* base = pk.rbuf[m];
        if (!base) {  // (the window that only drains the carry)
            pk.text[m].resize_uninit((size_t)pk.rccap + 16);
            base = pk.text[m].data();
        }
        if (pk.rcin[m]) {
            if (!prev.buf[m] || prev.end[m] < pk.rcin[m]) throw std::runtime_error("raw pack: carry without its window");
            std::memcpy(base + pk.rccap - pk.rcin[m], prev.buf[m] + prev.end[m] - pk.rcin[m], (size_t)pk.rcin[m]);
        }
        pk.base[m] = base;
    }
    std::shared_ptr<void> hold;  // (the last owner returns the window to the reader)
    if (pk.stage >= 0 && pk.stage_release)
        hold = std::shared_ptr<void>(nullptr, [rel = pk.stage_release, st = pk.stage](void*) { rel(st); });
    pk.stage = -1;
    prev.hold = hold;  // (the previous window goes back here, unless its writers still hold it)
    pk.zc = zc;
    if (zc) pk.hold = hold;
    for (int m = 0; m < mates; ++m) {
        prev.buf[m] = const_cast<char*>(pk.base[m]);
        prev.end[m] = pk.rccap + pk.rwin[m];
    }
    const size_t n = (size_t)pk.n;
    const fq_read_result* res = pk.res.data();
    auto passes = [](const fq_read_result& r) {
        return !(r.flags & (FQ_RF_NULL | FQ_RF_INDEX_FILTERED)) && r.code == FQ_PASS_FILTER;
    };
    auto out_ok = [&](size_t i) {
        return pk.paired ? passes(res[2 * i]) && passes(res[2 * i + 1]) : passes(res[i]);
    };
    auto rr = [&](size_t i, int m) -> const fq_read_result& { return res[pk.paired ? 2 * i + m : i]; };
    auto entry_bytes = [](const fq_read_result& r) -> size_t {
        if (!(r.flags & (FQ_RF_AD_OVERLAP | FQ_RF_AD_SEQ)) || r.ad_len == 0) return 0;
        return (r.flags & FQ_RF_AD_NEG) ? 5 : 3 + (size_t)r.ad_len;
    };
    const int parts = std::max(1, std::min(pool.size() * 2, (int)((n + 4095) / 4096)));
    std::vector<size_t> osz((size_t)parts * 2, 0), esz((size_t)parts * 2, 0);
    auto untrimmed = [](const fq_text_rec& R, const fq_read_result& r) { return r.start == 0 && r.len == R.len; };
    pool.run(parts, [&](int k) {
        const size_t i0 = n * (size_t)k / (size_t)parts, i1 = n * (size_t)(k + 1) / (size_t)parts;
        for (int m = 0; m < mates; ++m) {
            const fq_text_rec* T = pk.trec[m].data();
            size_t o = 0, e = 0;
            for (size_t i = i0; i < i1; ++i) {
                const fq_read_result& r = rr(i, m);
                if (out_ok(i) && !(zc && untrimmed(T[i], r))) o += (size_t)T[i].name_len + T[i].strand_len + 2 * (size_t)r.len + 4;
                if (adapters) e += entry_bytes(r);
            }
            osz[(size_t)(2 * k + m)] = o;
            esz[(size_t)(2 * k + m)] = e;
        }
    });
    size_t otot[2] = {0, 0}, etot[2] = {0, 0};
    for (int k = 0; k < parts; ++k)
        for (int m = 0; m < mates; ++m) {
            const size_t a = osz[(size_t)(2 * k + m)], b = esz[(size_t)(2 * k + m)];
            osz[(size_t)(2 * k + m)] = otot[m];
            esz[(size_t)(2 * k + m)] = etot[m];
            otot[m] += a;
            etot[m] += b;
        }
    for (int m = 0; m < mates; ++m) {
        pk.out_text[m].resize_uninit(otot[m] + etot[m] + 16);
        pk.tout.text[m] = pk.out_text[m].data();
        pk.tout.bytes[m] = otot[m];
    }
    std::vector<std::vector<iovec>> psegs(zc ? (size_t)parts * 2 : 0);
    pool.run(parts, [&](int k) {
        const size_t i0 = n * (size_t)k / (size_t)parts, i1 = n * (size_t)(k + 1) / (size_t)parts;
        for (int m = 0; m < mates; ++m) {
            const fq_text_rec* T = pk.trec[m].data();
            const char* t = pk.base[m];
            char* d = pk.out_text[m].data() + osz[(size_t)(2 * k + m)];
            char* ed = pk.out_text[m].data() + otot[m] + esz[(size_t)(2 * k + m)];
            std::vector<iovec>* sg = zc ? &psegs[(size_t)(2 * k + m)] : nullptr;
            auto range = [sg](const char* a, size_t len) {  // (contiguous with the last range: one range)
                if (!sg->empty() && static_cast<const char*>(sg->back().iov_base) + sg->back().iov_len == a)
                    sg->back().iov_len += len;
                else
                    sg->push_back(iovec{const_cast<char*>(a), len});
            };
            for (size_t i = i0; i < i1; ++i) {
                const fq_text_rec& R = T[i];
                const fq_read_result& r = rr(i, m);
                const char* d0 = d;
                if (out_ok(i) && untrimmed(R, r)) {
                    // an untrimmed record is its input text as it stands (raw records are "plain":
                    // four lines, each ending in '\n'): one copy, or (zc) a range of the window
                    const size_t nb = (size_t)R.name_len + R.strand_len + 2 * (size_t)R.len + 4;
                    if (zc) {
                        range(t + R.name_off, nb);
                    } else {
                        std::memcpy(d, t + R.name_off, nb);
                        d += nb;
                    }
                } else if (out_ok(i)) {
                    std::memcpy(d, t + R.name_off, R.name_len);
                    d += R.name_len;
                    *d++ = '\n';
                    std::memcpy(d, t + R.seq_off + r.start, r.len);
                    d += r.len;
                    *d++ = '\n';
                    std::memcpy(d, t + R.strand_off, R.strand_len);
                    d += R.strand_len;
                    *d++ = '\n';
                    std::memcpy(d, t + R.qual_off + r.start, r.len);
                    d += r.len;
                    *d++ = '\n';
                    if (zc) range(d0, (size_t)(d - d0));
                }
                if (adapters && entry_bytes(r)) {
                    ed[0] = (char)(r.ad_len & 0xFF);
                    ed[1] = (char)(r.ad_len >> 8);
                    if (r.flags & FQ_RF_AD_NEG) {
                        ed[2] = 1;
                        ed[3] = (char)(r.ad_pos & 0xFF);
                        ed[4] = (char)(r.ad_pos >> 8);
                        ed += 5;
                    } else {
                        ed[2] = 0;
                        std::memcpy(ed + 3, t + R.seq_off + r.ad_pos, r.ad_len);
                        ed += 3 + r.ad_len;
                    }
                }
            }
        }
    });
    if (zc)
        for (int m = 0; m < mates; ++m) {
            std::vector<iovec>& v = pk.segs[m];
            v.clear();
            for (int k = 0; k < parts; ++k)
                for (const iovec& x : psegs[(size_t)(2 * k + m)]) {
                    if (!v.empty() && static_cast<char*>(v.back().iov_base) + v.back().iov_len == x.iov_base)
                        v.back().iov_len += x.iov_len;
                    else
                        v.push_back(x);
                }
        }
    if (adapters)
        for (int m = 0; m < mates; ++m) ac.add_entries(m, pk.out_text[m].data() + otot[m], etot[m], p, &pool);
}

// Raw streams on several engines (--devices with more than one entry; fq_engine_raw_*).  The host cuts
// the inputs into windows of whole pairs: it counts the line feeds of the bytes it preads and ends
// every mate's window after the same number of four-line records (at most the engines' max_batch),
// so the windows are independent of each other and go round-robin to the engines (window k to
// engine k mod G, pack seq_no k), each engine copying, indexing and running its own.  A window's
// pack launches only after the window before it has launched and taken all its pairs (the GPU's
// indexing reports that at launch, fq_raw_result), so when the GPU path stops -- an irregular record
// the line count could not see (empty or '\r'-ended lines, a read longer than the engine takes) --
// no later window has reached a kernel or an accumulator: the engines drop the windows they hold and
// the host reader resumes at the stopping window's offsets, pack numbers continuing (as with one
// engine, src/fqreader.cpp:160-195).
struct RawStage {  // one window's page-locked staging (one buffer per mate)
    RawStage() : buf{ByteBuf(true), ByteBuf(true)} {}
    ByteBuf buf[2];
};
struct RawResumeInfo {
    bool done = false;
    uint64_t off[2] = {0, 0};
    uint64_t next_seq = 0;
};
struct RawMulti {
    struct Win {
        uint64_t id = 0, start[2] = {0, 0}, n[2] = {0, 0};
        int64_t pairs = 0;
        int stage = -1;
        bool end = false;  // no window: the stream ends here (the host reader takes start[])
    };
    int G = 1, mates = 1;
    int fd[2] = {-1, -1};
    uint64_t size[2] = {0, 0};
    uint64_t wcap = (uint64_t)48 << 20;
    std::vector<std::unique_ptr<RawStage>> stages;
    Queue<int> free_stages{1024};
    std::vector<std::unique_ptr<Queue<Win>>> wq;  // per engine, windows in id order
    std::mutex m;
    std::condition_variable cv;
    uint64_t next_launch = 0;  // the id allowed to launch next
    uint64_t next_enqueue = 0;  // the id allowed to enqueue next (its copies follow the previous
                                // window's on a shared GPU: fq_engine_raw_enqueue)
    bool stopped = false;      // the stream has ended; rr says where
    RawResumeInfo rr;
    std::string why;
    std::atomic<uint64_t> pairs{0}, packs{0};
    double read_s = 0, stage_wait_s = 0;
    std::exception_ptr err;
    std::function<void(const RawResumeInfo&)> on_end;  // called once, when `stopped` is set

    ~RawMulti() {
        for (int& f : fd)
            if (f >= 0) ::close(f);
    }
    // under m: the stream ends (first caller wins)
    void end_locked(const RawResumeInfo& r, const std::string& w) {
        if (stopped) return;
        stopped = true;
        rr = r;
        why = w;
        cv.notify_all();
        free_stages.close();  // (the window reader stops at its next stage)
        if (on_end) on_end(rr);
    }
    void fail(std::exception_ptr e) {
        std::lock_guard<std::mutex> g(m);
        if (!err) err = e;
        RawResumeInfo r;  // (the caller rethrows; the host reader must not wait forever, nor read)
        r.done = true;
        end_locked(r, "error");
    }

    // The window reader: exact pair-aligned windows, dealt round-robin; runs until the input is
    // consumed, a window cannot be cut, or the stream stopped.
    void read_windows(int target, int max_batch, Pool& pool) {
        try {
            uint64_t pos[2] = {0, 0};
            double bpr[2] = {0, 0};  // bytes per record so far
            const uint64_t piece = (uint64_t)1 << 20;
            const char* w0_env = std::getenv("FQ_RAW_WINDOW0");  // first window's bytes (tests: tiny windows)
            const uint64_t w0 = w0_env ? std::max<uint64_t>(4096, std::strtoull(w0_env, nullptr, 10)) : (uint64_t)4 << 20;
            std::vector<uint32_t> cnt[2];
            for (uint64_t id = 0;; ++id) {
                {
                    std::lock_guard<std::mutex> g(m);
                    if (stopped) break;
                }
                Win w;
                w.id = id;
                bool left = false;
                for (int k = 0; k < mates; ++k) left = left || pos[k] < size[k];
                if (!left) {
                    w.end = true;
                    for (int k = 0; k < mates; ++k) w.start[k] = pos[k];
                    wq[(size_t)(id % (uint64_t)G)]->push(w);
                    break;
                }
                const auto s0 = std::chrono::steady_clock::now();
                if (!free_stages.pop(w.stage)) break;
                stage_wait_s += since(s0);
                RawStage& st = *stages[(size_t)w.stage];
                uint64_t want[2] = {0, 0};
                for (int k = 0; k < mates; ++k)
                    want[k] = bpr[k] > 0 ? (uint64_t)(target * bpr[k] * 1.02) + 4096 : w0;
                int64_t P = 0;
                for (;;) {  // read, count records; grow the window when it holds no whole pair
                    const auto r0 = std::chrono::steady_clock::now();
                    uint64_t n[2] = {0, 0};
                    int pieces[2] = {0, 0};
                    for (int k = 0; k < mates; ++k) {
                        n[k] = std::min(std::min(want[k], wcap), size[k] - pos[k]);
                        st.buf[k].resize_uninit((size_t)std::max<uint64_t>(n[k], 1));
                        pieces[k] = (int)((n[k] + piece - 1) / piece);
                        cnt[k].assign((size_t)pieces[k], 0);
                    }
                    std::atomic<bool> short_read{false};
                    pool.run(pieces[0] + pieces[1], [&](int q) {
                        const int k = q < pieces[0] ? 0 : 1;
                        const int pi = k ? q - pieces[0] : q;
                        const uint64_t o = (uint64_t)pi * piece, len = std::min(piece, n[k] - o);
                        char* dst = st.buf[k].data() + o;
                        uint64_t got = 0;
                        while (got < len) {
                            const ssize_t r = pread(fd[k], dst + got, (size_t)(len - got), (off_t)(pos[k] + o + got));
                            if (r <= 0) {
                                short_read = true;
                                return;
                            }
                            got += (uint64_t)r;
                        }
                        cnt[k][(size_t)pi] = count_lf(dst, (size_t)len);
                    });
                    if (short_read) throw std::runtime_error("input file changed while reading");
                    read_s += since(r0);
                    P = max_batch;
                    for (int k = 0; k < mates; ++k) {
                        uint64_t lf = 0;
                        for (uint32_t c : cnt[k]) lf += c;
                        P = std::min<int64_t>(P, (int64_t)(lf / 4));
                    }
                    bool can_grow = false;
                    for (int k = 0; k < mates; ++k) can_grow = can_grow || (n[k] < wcap && pos[k] + n[k] < size[k]);
                    if (P > 0 || !can_grow) {
                        for (int k = 0; k < mates; ++k) w.n[k] = n[k];
                        break;
                    }
                    for (int k = 0; k < mates; ++k) want[k] = std::min(wcap, std::max<uint64_t>(2 * n[k], 4096));
                }
                if (P <= 0) {  // no whole pair fits: the host reader takes it from here
                    free_stages.push(w.stage);
                    w.stage = -1;
                    w.end = true;
                    for (int k = 0; k < mates; ++k) {
                        w.start[k] = pos[k];
                        w.n[k] = 0;
                    }
                    wq[(size_t)(id % (uint64_t)G)]->push(w);
                    break;
                }
                for (int k = 0; k < mates; ++k) {  // each mate's window ends after its P-th record
                    const uint64_t target_lf = 4 * (uint64_t)P;
                    uint64_t seen = 0;
                    size_t pi = 0;
                    while (seen + cnt[k][pi] < target_lf) seen += cnt[k][pi++];
                    const uint64_t at = nth_lf(st.buf[k].data() + pi * piece, (size_t)std::min(piece, w.n[k] - pi * piece),
                                               (size_t)(target_lf - seen));
                    w.start[k] = pos[k];
                    w.n[k] = pi * piece + at + 1;
                    pos[k] += w.n[k];
                    bpr[k] = bpr[k] > 0 ? 0.5 * bpr[k] + 0.5 * (double)w.n[k] / (double)P : (double)w.n[k] / (double)P;
                }
                w.pairs = P;
                if (!wq[(size_t)(id % (uint64_t)G)]->push(w)) {
                    free_stages.push(w.stage);
                    break;
                }
            }
        } catch (...) {
            fail(std::current_exception());
        }
        for (auto& q : wq) q->close();
    }
    // Line feeds in [p, p + n): byte counters (each compare's 0xFF subtracted, i.e. +1), summed by
    // v_sad-style _mm_sad_epu8 every 255 steps -- no popcount (the build targets baseline x86-64,
    // where __builtin_popcount is a library call per 16 bytes).
    static uint32_t count_lf(const char* p, size_t n) {
        // (32 bytes a step where the CPU has AVX2 -- the build targets baseline x86-64, so the wider
        // loop is compiled for it alone and picked at run time)
        static const bool avx2 = __builtin_cpu_supports("avx2");
        if (avx2) return count_lf_avx2(p, n);
        uint64_t c = 0;
        size_t i = 0;
        const __m128i nl = _mm_set1_epi8('\n'), zero = _mm_setzero_si128();
        while (i + 16 <= n) {
            __m128i acc = zero;
            const size_t end = std::min(n & ~(size_t)15, i + 255 * 16);
            for (; i < end; i += 16)
                acc = _mm_sub_epi8(acc, _mm_cmpeq_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p + i)), nl));
            const __m128i s = _mm_sad_epu8(acc, zero);
            c += (uint64_t)_mm_cvtsi128_si64(s) + (uint64_t)_mm_cvtsi128_si64(_mm_unpackhi_epi64(s, s));
        }
        for (; i < n; ++i) c += p[i] == '\n';
        return (uint32_t)c;
    }
    __attribute__((target("avx2"))) static uint32_t count_lf_avx2(const char* p, size_t n) {
        uint64_t c = 0;
        size_t i = 0;
        const __m256i nl = _mm256_set1_epi8('\n'), zero = _mm256_setzero_si256();
        while (i + 64 <= n) {  // two byte-counter vectors, 64 bytes a step, summed every 255 steps
            __m256i a0 = zero, a1 = zero;
            const size_t end = std::min(n & ~(size_t)63, i + 255 * 64);
            for (; i < end; i += 64) {
                a0 = _mm256_sub_epi8(a0, _mm256_cmpeq_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(p + i)), nl));
                a1 = _mm256_sub_epi8(a1, _mm256_cmpeq_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(p + i + 32)), nl));
            }
            const __m256i s = _mm256_add_epi64(_mm256_sad_epu8(a0, zero), _mm256_sad_epu8(a1, zero));
            c += (uint64_t)_mm256_extract_epi64(s, 0) + (uint64_t)_mm256_extract_epi64(s, 1) +
                 (uint64_t)_mm256_extract_epi64(s, 2) + (uint64_t)_mm256_extract_epi64(s, 3);
        }
        for (; i < n; ++i) c += p[i] == '\n';
        return (uint32_t)c;
    }
    // offset of the k-th (1-based) line feed in [p, p + n): whole 4 KiB blocks counted as above, then
    // 16 bytes a step within the block that holds it
    static uint64_t nth_lf(const char* p, size_t n, size_t k) {
        size_t b = 0;
        for (; b + 4096 <= n; b += 4096) {
            const size_t c = count_lf(p + b, 4096);
            if (c >= k) break;
            k -= c;
        }
        return b + nth_lf_scan(p + b, n - b, k);
    }
    static uint64_t nth_lf_scan(const char* p, size_t n, size_t k) {
        size_t i = 0;
        const __m128i nl = _mm_set1_epi8('\n');
        for (; i + 16 <= n; i += 16) {  // 16 bytes a step; the k-th within a step by its bit mask
            unsigned mk = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p + i)), nl));
            const size_t c = (size_t)popcount16(mk);
            if (c < k) {
                k -= c;
                continue;
            }
            while (--k) mk &= mk - 1;
            return i + (uint64_t)__builtin_ctz(mk);
        }
        for (; i < n; ++i)
            if (p[i] == '\n' && --k == 0) return i;
        throw std::runtime_error("raw window: line feed count mismatch");
    }
    static unsigned popcount16(unsigned x) {  // (16-bit mask; baseline x86-64 has no popcnt)
        x = x - ((x >> 1) & 0x5555u);
        x = (x & 0x3333u) + ((x >> 2) & 0x3333u);
        x = (x + (x >> 4)) & 0x0F0Fu;
        return (x + (x >> 8)) & 0x1Fu;
    }
};

// One engine per entry of --devices (several may share a GPU), each fed by its own dispatcher
// thread: pack k goes to engine k mod G.  A pack with longer reads (or more of them) re-creates
// that engine larger after draining it.
struct Lane {
    Lane(int device, int depth_) : dev(device), depth(depth_), in(2), out((size_t)depth_ + 2) {}
    ~Lane() {
        if (t.joinable()) t.join();
        if (e) fq_engine_destroy(e);
        if (dup) fq_dup_destroy(dup);
    }
    int dev, depth;
    fq_engine* e = nullptr;
    fq_dup* dup = nullptr;  // -d: this engine's table, kept across re-creation
    int max_cycles = 0, max_batch = 0, max_stride = 0;
    Queue<std::unique_ptr<Pack>> in, out;
    std::deque<std::unique_ptr<Pack>> inflight;  // submission order == input order
    std::thread t;
    std::exception_ptr err;
    double tiles_s = 0, submit_s = 0, wait_s = 0;
    double first_submit = -1;  // seconds from t_start to this engine's first submission
    std::chrono::steady_clock::time_point t_start = std::chrono::steady_clock::now();

    void make(const Options& o, int cycles, int batch, int stride) {
        if (e) fq_engine_destroy(e);
        e = nullptr;
        fq_params p = o.to_params(cycles);
        if (fq_engine_create(&p, dev, batch, stride, &e) != FQ_OK)
            throw std::runtime_error("fq_engine_create (device " + std::to_string(dev) + "): " + fq_engine_last_error(nullptr));
        if (o.dup) {
            if (!dup && fq_dup_create(dev, o.dup_keylen, &dup) != FQ_OK)
                throw std::runtime_error("fq_dup_create (device " + std::to_string(dev) + ") failed");
            if (fq_engine_set_dup(e, dup) != FQ_OK)
                throw std::runtime_error(std::string("fq_engine_set_dup: ") + fq_engine_last_error(e));
        }
        max_cycles = cycles;
        max_batch = batch;
        max_stride = stride;
    }

    // the engine's accumulators summed into the host's (RCCL-free: they are in this process)
    void drain(HostAcc& acc) {
        std::vector<uint64_t> buf(fq_engine_acc_words(e));
        if (fq_engine_read_acc(e, buf.data(), buf.size()) != FQ_OK)
            throw std::runtime_error(std::string("fq_engine_read_acc: ") + fq_engine_last_error(e));
        acc.add(buf.data(), max_cycles);
        fq_engine_reset_acc(e);
    }

    // the oldest pack in flight, once complete, to the formatter; wait == false: only if it is done
    bool complete_oldest(bool wait = true) {
        uint64_t seq = 0;
        const auto e0 = std::chrono::steady_clock::now();
        const int rc = fq_engine_poll(e, wait ? 1 : 0, &seq);
        wait_s += since(e0);
        if (rc == 0 && !wait) return false;
        std::unique_ptr<Pack> pk = std::move(inflight.front());
        inflight.pop_front();
        if (rc != 1) throw std::runtime_error(std::string("fq_engine_poll: ") + fq_engine_last_error(e));
        if (seq != pk->seq_no) throw std::runtime_error("engine completed packs out of order");
        if (pk->raw) {  // its input window was copied: recycle the staging; the output sizes are in
            // (records-only egress: the formatter still reads the window, and returns it)
            if (pk->stage >= 0 && !pk->recs) (multi ? multi->free_stages : free_stages).push(pk->stage);
            if (!pk->recs) pk->stage = -1;
            pk->tout = pk->rout.text;
        }
        if (!out.push(std::move(pk))) throw Stopped();
        return true;
    }

    void submit(Pack& pk, bool as_text) {
        const auto e0 = std::chrono::steady_clock::now();
        if (as_text) {
            fq_text_batch tb{};
            tb.n = pk.n;
            tb.stride = pk.stride;
            for (int m = 0; m < (pk.paired ? 2 : 1); ++m) {
                tb.text[m] = pk.span[m];
                tb.text_bytes[m] = pk.span_bytes[m];
                tb.rec[m] = pk.trec[m].data();
            }
            if (fq_engine_submit_text(e, &tb, pk.results(), &pk.tout, pk.seq_no) != FQ_OK)
                throw std::runtime_error(std::string("fq_engine_submit_text: ") + fq_engine_last_error(e));
        } else {
            const fq_batch b = pk.batch();
            if (fq_engine_submit(e, &b, pk.results(), pk.seq_no) != FQ_OK)
                throw std::runtime_error(std::string("fq_engine_submit: ") + fq_engine_last_error(e));
        }
        submit_s += since(e0);
    }

    // Raw-stream ingest (fq_engine_raw_*, include/fqengine.h): the inputs (regular files) go to
    // the GPU in consecutive windows; the engine cuts the records, pairs the mates and runs the
    // pack.  A reader thread fills page-locked staging windows with parallel preads on the pool
    // (no mapping, no registration: the copies are plain DMA) while this thread enqueues them and
    // launches the packs.  Windows are sized to bring about `target` pairs per pack from what the
    // packs so far took per pair and left over (published after every launch).  Ends at the end
    // of the input (done) or where the GPU path stops (an irregular record, no progress, bytes
    // left at the end): the host reader then resumes at the returned stream offsets, pack numbers
    // continuing.
    struct RawResume {
        bool done = false;
        uint64_t off[2] = {0, 0};
        uint64_t next_seq = 0;
    };
    struct Stage {  // one window's staging buffers (one per mate)
        Stage() : buf{ByteBuf(true), ByteBuf(true)} {}
        ByteBuf buf[2];
    };
    std::vector<std::unique_ptr<Stage>> stages;
    Queue<int> free_stages{64};
    RawMulti* multi = nullptr;  // several engines: the shared window source (run_raw_multi)
    bool merge = false;         // -m (PE): raw packs' mate-0 output is the merged stream
    uint64_t raw_pairs = 0, raw_packs = 0;  // what the raw stream took
    double raw_read_s = 0, raw_stage_wait_s = 0, raw_ready_wait_s = 0;  // window reader: preads, waits
    double raw_pack_wait_s = 0, raw_enqueue_s = 0;  // dispatcher: waiting for a spare pack, enqueue calls
    double raw_turn_wait_s = 0, raw_idx_wait_s = 0;  // several engines: waiting for the turn, for the own index
    std::string raw_end;                    // why it ended
    std::unique_ptr<ParGzSource> pre_gz[2];  // gzip inputs' inflaters, started ahead of the engines

    RawResume run_raw(const std::string* files, int mates, int target, int est_len, Queue<std::unique_ptr<Pack>>& spare, Pool& pool) {
        RawResume rr;
        int fd[2] = {-1, -1};
        uint64_t size[2] = {0, 0};
        auto close_all = [&] {
            for (int& f : fd)
                if (f >= 0) {
                    ::close(f);
                    f = -1;
                }
        };
        // single-stream gzip inputs: each mate's stream comes from its parallel inflater, in order
        // (the windows are consecutive); its size is known once the inflater ends it.  A stream
        // that fails (corrupt data) ends the raw stream short of the bad call: the host reader
        // then resumes there and meets the failure as the reference's reader does.
        std::unique_ptr<ParGzSource> gzs[2];
        std::atomic<bool> src_failed{false};
        const bool gz_in = ends_with_gz(files[0]);
        for (int m = 0; m < mates; ++m) {
            if (gz_in) {
                // (opened, and inflating, before the engines were made: run_tool)
                gzs[m] = pre_gz[m] ? std::move(pre_gz[m]) : ParGzSource::open(files[m], (size_t)1 << 20, gz_inflate_threads());
                if (!gzs[m]) return rr;  // (the host reader takes the whole input)
                size[m] = UINT64_MAX;
                continue;
            }
            fd[m] = ::open(files[m].c_str(), O_RDONLY);
            struct stat st;
            if (fd[m] < 0 || fstat(fd[m], &st) != 0 || !S_ISREG(st.st_mode) || st.st_size <= 0) {
                close_all();
                return rr;  // (the host reader takes the whole input)
            }
            size[m] = (uint64_t)st.st_size;
            (void)posix_fadvise(fd[m], 0, 0, POSIX_FADV_SEQUENTIAL);
        }
        // windows of up to 48 MiB per mate (a pack of `target` 2x150 pairs is ~45 MiB; longer reads
        // make smaller packs: every page-locked byte costs ~40 ms/GiB again when the process exits,
        // tools/micro/exit_cost), 16 MiB of
        // carry (partial records, the mates' imbalance); six windows in the engine at once
        // (smaller packs, --pack_pairs: windows of ~1.3 packs of the estimated record size, so the
        // page-locked stages shrink with them)
        const uint64_t rec_est = 2 * (uint64_t)std::max(est_len, 16) + 72;
        const uint64_t wfit = ((uint64_t)(1.3 * (double)target * (double)rec_est) + ((uint64_t)1 << 20)) & ~(((uint64_t)1 << 20) - 1);
        const uint64_t wcap = std::min<uint64_t>((uint64_t)48 << 20, std::max<uint64_t>((uint64_t)4 << 20, wfit));
        const uint64_t ccap = (uint64_t)16 << 20;
        // records-only egress (FQ_RAW_EGRESS=host): the engine sends back records and line offsets,
        // the formatter writes the output from the staging window, which then keeps the carry
        // capacity free in front of the window bytes (the device buffer's layout)
        const char* eg_env = std::getenv("FQ_RAW_EGRESS");
        const bool recs = !merge && eg_env && std::string(eg_env) == "host";
        const uint64_t off0 = recs ? ccap : 0;
        const int raw_depth = 4;  // packs launched and not yet polled
        const size_t raw_ahead = 3;  // windows enqueued ahead of their launch (the copy-in queue)
        if (fq_engine_raw_begin(e, wcap, ccap) != FQ_OK)
            throw std::runtime_error(std::string("fq_engine_raw_begin: ") + fq_engine_last_error(e));
        // in flight + enqueued + being filled, and one more so the window reader can run ahead of
        // the packs (a stage comes back only when its pack completes).  Ten stages ran the 50 M-pair
        // pipeline as fast as thirteen (0.78-0.87 s vs 0.80-0.85 s) with ~0.3 GiB less page-locked
        // memory to release at the exit (profiles/r04_e2e_stages_10_13.txt)
        const char* st_env = std::getenv("FQ_RAW_STAGES");  // (profiling)
        const int kStages = std::max(raw_depth + (int)raw_ahead + 2, st_env ? std::atoi(st_env) : raw_depth + (int)raw_ahead + 3);
        // The first new stage is handed out at once; the others are made page-locked (~0.06 s/GiB)
        // on a helper thread and handed out as they become ready, so their registration overlaps
        // the first windows instead of stalling the reader.
        std::thread warmer;
        struct Joiner {
            std::thread& t;
            ~Joiner() {
                if (t.joinable()) t.join();
            }
        } warmer_join{warmer};
        if ((int)stages.size() < kStages) {
            const int have = (int)stages.size();
            while ((int)stages.size() < kStages) stages.emplace_back(new Stage);
            free_stages.push(have);
            warmer = std::thread([this, have, kStages, wcap, off0, mates] {
                try {
                    for (int i = have + 1; i < kStages; ++i) {
                        for (int m = 0; m < mates; ++m) stages[(size_t)i]->buf[m].reserve((size_t)(off0 + wcap));
                        if (!free_stages.push(i)) break;
                    }
                } catch (...) {  // (no page-locked memory left: the stages made so far suffice)
                }
            });
        }
        struct Win {
            uint64_t start[2] = {0, 0}, n[2] = {0, 0};
            int stage = -1;
            uint64_t id = 0;
        };
        // published by this thread after each launch, read by the window reader
        std::mutex fb_m;
        double bpr[2] = {0, 0};      // text bytes per record of the packs so far
        uint64_t carry[2] = {0, 0};  // after the last launched window
        uint64_t launched = 0;       // windows launched
        Queue<Win> ready(3);
        std::exception_ptr rd_err;
        const char* pc_env = std::getenv("FQ_RAW_PIECE_MB");  // (profiling: pread piece size)
        const uint64_t piece_bytes = (uint64_t)(pc_env ? std::max(1, atoi(pc_env)) : 1) << 20;
        const char* cp_env = std::getenv("FQ_RAW_COPY");
        const char* mp[2] = {nullptr, nullptr};
        if (cp_env && std::string(cp_env) == "mmap")
            for (int m = 0; m < mates; ++m) {
                void* a = mmap(nullptr, (size_t)size[m], PROT_READ, MAP_PRIVATE, fd[m], 0);
                if (a != MAP_FAILED) {
                    madvise(a, (size_t)size[m], MADV_SEQUENTIAL);
                    mp[m] = static_cast<const char*>(a);
                }
            }
        const char* w0_env = std::getenv("FQ_RAW_WINDOW0");  // first window's bytes (tests: tiny windows)
        const uint64_t w0 = w0_env ? std::max<uint64_t>(4096, std::strtoull(w0_env, nullptr, 10)) : (uint64_t)4 << 20;
        std::thread rd([&] {  // the window reader
            try {
                uint64_t pos[2] = {0, 0};
                uint64_t rsize[2] = {size[0], size[1]};  // (this thread's copy: a gzip stream's grows known)
                std::deque<Win> made;  // windows produced and (maybe) not yet launched
                for (uint64_t id = 0;; ++id) {
                    bool more = false;
                    for (int m = 0; m < mates; ++m) more = more || pos[m] < rsize[m];
                    if (!more) break;
                    double b[2], pairs_held = 1e18;
                    uint64_t held[2];
                    {
                        std::lock_guard<std::mutex> g(fb_m);
                        while (!made.empty() && made.front().id < launched) made.pop_front();
                        for (int m = 0; m < 2; ++m) {
                            b[m] = bpr[m];
                            held[m] = carry[m];
                        }
                    }
                    for (const Win& q : made)
                        for (int m = 0; m < mates; ++m) held[m] += q.n[m];
                    for (int m = 0; m < mates; ++m) pairs_held = std::min(pairs_held, b[m] > 0 ? held[m] / b[m] : 0.0);
                    // the packs of the windows still queued take up to `target` pairs each before
                    // this window's pack: what they leave over is the new window's carry
                    const double queued_pairs = (double)target * (double)made.size();
                    Win w;
                    w.id = id;
                    for (int m = 0; m < mates; ++m) {
                        uint64_t want;
                        if (b[m] <= 0) {
                            want = w0;
                        } else {
                            const double after = held[m] - std::min(pairs_held, queued_pairs) * b[m];
                            const double need = target * b[m] * 1.02 - std::max(0.0, after);
                            want = need <= 0 ? 0 : (uint64_t)need;
                        }
                        w.start[m] = pos[m];
                        w.n[m] = std::min(std::min<uint64_t>((want + 4095) / 4096 * 4096, wcap), rsize[m] - pos[m]);
                        pos[m] += w.n[m];
                    }
                    const auto s0 = std::chrono::steady_clock::now();
                    if (!free_stages.pop(w.stage)) break;
                    raw_stage_wait_s += since(s0);
                    const auto r0 = std::chrono::steady_clock::now();
                    Stage& st = *stages[(size_t)w.stage];
                    const uint64_t piece = piece_bytes;
                    int pieces[2] = {0, 0};
                    for (int m = 0; m < mates; ++m) {
                        st.buf[m].resize_uninit((size_t)(off0 + std::max<uint64_t>(w.n[m], 1)));
                        pieces[m] = (int)((w.n[m] + piece - 1) / piece);
                    }
                    std::atomic<bool> short_read{false};
                    if (gz_in) {
                        // the mates' streams are read side by side (each read copies its bytes out of
                        // the inflater's chunks: one thread for both would serialise the copies)
                        size_t got[2] = {0, 0};
                        bool bad[2] = {false, false};
                        pool.run(mates, [&](int m) {
                            if (w.n[m]) bad[m] = !gzs[m]->read(st.buf[m].data() + off0, (size_t)w.n[m], got[m]);
                        });
                        bool ended = true;
                        for (int m = 0; m < mates; ++m) {
                            if (bad[m]) src_failed = true;
                            if (got[m] < w.n[m]) {  // the stream's end (or its failure)
                                w.n[m] = got[m];
                                pos[m] = w.start[m] + got[m];
                                rsize[m] = pos[m];
                                std::lock_guard<std::mutex> g(fb_m);
                                size[m] = rsize[m];
                            }
                            ended = ended && w.n[m] == 0 && pos[m] == rsize[m];
                        }
                        pieces[0] = pieces[1] = 0;
                        if (ended) {  // (every stream has ended: no window)
                            free_stages.push(w.stage);
                            break;
                        }
                    }
                    pool.run(pieces[0] + pieces[1], [&](int k) {
                        const int m = k < pieces[0] ? 0 : 1;
                        const uint64_t o = (uint64_t)(m ? k - pieces[0] : k) * piece;
                        const uint64_t len = std::min(piece, w.n[m] - o);
                        char* dst = st.buf[m].data() + off0 + o;
                        if (mp[m]) {  // (FQ_RAW_COPY=mmap: copy from a read-only mapping)
                            std::memcpy(dst, mp[m] + w.start[m] + o, (size_t)len);
                            return;
                        }
                        uint64_t got = 0;
                        while (got < len) {
                            const ssize_t r = pread(fd[m], dst + got, (size_t)(len - got), (off_t)(w.start[m] + o + got));
                            if (r <= 0) {
                                short_read = true;
                                return;
                            }
                            got += (uint64_t)r;
                        }
                    });
                    if (short_read) throw std::runtime_error("input file changed while reading");
                    raw_read_s += since(r0);
                    made.push_back(w);
                    if (!ready.push(w)) break;
                    if (src_failed) break;  // (no window past a failed gzip read)
                }
            } catch (...) {
                rd_err = std::current_exception();
            }
            ready.close();
        });
        std::deque<Win> wins;  // enqueued, not launched
        bool input_done = false;
        auto enqueue_window = [&](const Win& w) {  // (stage -1: an empty window)
            fq_raw_window rw{};
            for (int m = 0; m < mates; ++m) {
                rw.bytes[m] = w.stage >= 0 ? stages[(size_t)w.stage]->buf[m].data() + off0 : nullptr;
                rw.n[m] = w.n[m];
            }
            const auto q0 = std::chrono::steady_clock::now();
            const int qrc = fq_engine_raw_enqueue(e, &rw);
            raw_enqueue_s += since(q0);
            if (qrc != FQ_OK) {
                if (w.stage >= 0) free_stages.push(w.stage);
                throw std::runtime_error(std::string("fq_engine_raw_enqueue: ") + fq_engine_last_error(e));
            }
            wins.push_back(w);
        };
        auto enqueue_next = [&]() -> bool {
            Win w;
            const auto q0 = std::chrono::steady_clock::now();
            const bool got = !input_done && ready.pop(w);
            raw_ready_wait_s += since(q0);
            if (!got) {
                input_done = true;
                return false;
            }
            enqueue_window(w);
            return true;
        };
        uint64_t seq = 0;
        auto finish = [&] {
            ready.close();
            free_stages.close();  // (a reader waiting for a stage stops)
            rd.join();
            free_stages.reopen();
        };
        try {
            if (enqueue_next()) {
                for (;;) {
                    while (wins.size() < raw_ahead && enqueue_next()) {
                    }
                    const Win w = wins.front();
                    wins.pop_front();
                    std::unique_ptr<Pack> pk;
                    const auto p0 = std::chrono::steady_clock::now();
                    if (!spare.pop_recent(pk)) throw Stopped();
                    raw_pack_wait_s += since(p0);
                    pk->clear();
                    pk->raw = true;
                    pk->text_mode = true;
                    pk->paired = mates == 2;
                    pk->seq_no = seq;
                    pk->stage = w.stage;
                    uint64_t cin[2];
                    {
                        std::lock_guard<std::mutex> g(fb_m);
                        cin[0] = carry[0];
                        cin[1] = carry[1];
                    }
                    if (recs) {  // records and line offsets back; the formatter writes the text
                        pk->recs = true;
                        pk->rccap = ccap;
                        pk->stage_release = [this](int sidx) { free_stages.push(sidx); };
                        pk->res.resize((size_t)target * mates);
                        pk->rout.results = pk->res.data();
                        for (int m = 0; m < 2; ++m) {
                            pk->rbuf[m] = m < mates && w.stage >= 0 ? stages[(size_t)w.stage]->buf[m].data() : nullptr;
                            pk->rwin[m] = m < mates ? w.n[m] : 0;
                            pk->rcin[m] = m < mates ? cin[m] : 0;
                            if (m < mates) pk->trec[m].resize((size_t)target);
                            pk->rout.rec[m] = m < mates ? pk->trec[m].data() : nullptr;
                            pk->rout.text.text[m] = nullptr;
                        }
                    } else {
                        for (int m = 0; m < 2; ++m) {  // (output text, then the adapter entries)
                            size_t cap = m < mates ? (size_t)(cin[m] + w.n[m] + 4 * (uint64_t)target + 64) : 0;
                            if (merge && m == 0)  // (-m: the merged stream of both mates' text)
                                cap = (size_t)(cin[0] + w.n[0] + cin[1] + w.n[1] + 28 * (uint64_t)target + 64);
                            // (1/8 headroom when the page-locked buffer is first made or outgrown:
                            // windows vary by a few percent, and a regrowth registers anew)
                            pk->out_text[m].reserve(cap + cap / 8);
                            pk->out_text[m].resize_uninit(cap);
                            pk->rout.text.text[m] = m < mates ? pk->out_text[m].data() : nullptr;
                        }
                    }
                    fq_raw_result r{};
                    const auto e0 = std::chrono::steady_clock::now();
                    if (fq_engine_raw_launch(e, &r, &pk->rout, seq) != FQ_OK)
                        throw std::runtime_error(std::string("fq_engine_raw_launch: ") + fq_engine_last_error(e));
                    submit_s += since(e0);
                    if (first_submit < 0) first_submit = since(t_start);
                    pk->n = r.pairs;
                    pk->max_cycles = max_cycles;
                    {
                        std::lock_guard<std::mutex> g(fb_m);
                        for (int m = 0; m < mates; ++m) {
                            carry[m] = r.carry[m];
                            if (r.pairs > 0)
                                bpr[m] = bpr[m] > 0 ? 0.5 * bpr[m] + 0.5 * (double)r.text_bytes[m] / r.pairs
                                                    : (double)r.text_bytes[m] / r.pairs;
                        }
                        launched = w.id + 1;
                    }
                    // completed packs go on at once; wait only when the pipeline is full
                    while (!inflight.empty() && complete_oldest(false)) {
                    }
                    if ((int)inflight.size() >= raw_depth) complete_oldest();
                    inflight.push_back(std::move(pk));
                    ++seq;
                    if (wins.empty()) enqueue_next();
                    const bool last = wins.empty() && input_done;
                    const bool failed = src_failed;  // (a gzip input failed: its carry is not drained)
                    bool left = false, exhausted = false;  // (exhausted: a mate has sent all its bytes)
                    uint64_t sz_now[2];
                    {
                        std::lock_guard<std::mutex> g(fb_m);
                        sz_now[0] = size[0];
                        sz_now[1] = size[1];
                    }
                    for (int m = 0; m < mates; ++m) {
                        left = left || r.carry[m] > 0;
                        const uint64_t sent = wins.empty() ? w.start[m] + w.n[m] : wins.back().start[m] + wins.back().n[m];
                        exhausted = exhausted || sent == sz_now[m];
                    }
                    if (last && left && r.pairs > 0 && !r.stop && !failed) {  // all input is on the device: drain its carry
                        Win d;
                        for (int m = 0; m < mates; ++m) d.start[m] = sz_now[m];
                        enqueue_window(d);
                        raw_pairs += (uint64_t)r.pairs;
                        ++raw_packs;
                        continue;
                    }
                    raw_pairs += (uint64_t)r.pairs;
                    ++raw_packs;
                    // (no pairs while every mate still has bytes to send: the windows were too small)
                    if (r.stop || (r.pairs == 0 && exhausted) || last) {
                        rr.done = last && !left && !r.stop && !failed;
                        raw_end = rr.done ? "end of input"
                                          : std::string(r.stop ? "irregular record" : failed && last ? "gzip read failed ahead" : r.pairs == 0 ? "no pairs" : "bytes left at the end") +
                                                " after pack " + std::to_string(seq - 1) + " (window bytes " + std::to_string(w.n[0]) + "/" +
                                                std::to_string(w.n[1]) + ", carry " + std::to_string(r.carry[0]) + "/" +
                                                std::to_string(r.carry[1]) + ", max_len " + std::to_string(r.max_len) + ")";
                        for (int m = 0; m < mates; ++m) rr.off[m] = w.start[m] + w.n[m] - r.carry[m];
                        break;
                    }
                }
            } else {
                rr.done = false;  // (nothing to read: the host reader reports the empty input)
            }
            while (!inflight.empty()) complete_oldest();
            // windows enqueued after the stop are dropped once their copies are done, and the engine
            // leaves raw mode (the host reader's packs go to it next)
            (void)fq_engine_sync(e);
            if (fq_engine_raw_end(e) != FQ_OK)
                throw std::runtime_error(std::string("fq_engine_raw_end: ") + fq_engine_last_error(e));
            for (const Win& w : wins) free_stages.push(w.stage);
            wins.clear();
            finish();
            if (rd_err) std::rethrow_exception(rd_err);
        } catch (...) {
            (void)fq_engine_sync(e);
            (void)fq_engine_raw_end(e);
            inflight.clear();
            finish();
            close_all();
            throw;
        }
        close_all();
        for (int m = 0; m < mates; ++m)
            if (mp[m]) munmap(const_cast<char*>(mp[m]), (size_t)size[m]);
        rr.next_seq = seq;
        if (gz_in) raw_end += " (gzip inputs inflated on " + std::to_string(gz_inflate_threads()) + " threads each)";
        return rr;
    }

    // This engine's part of a raw stream on several engines (RawMulti): its windows in id order,
    // enqueued up to raw_ahead ahead, each launched in its turn (the previous window launched and
    // took all its pairs).
    void run_raw_multi(RawMulti& R, int g, int target, Queue<std::unique_ptr<Pack>>& spare) {
        multi = &R;
        const int raw_depth = 4;
        const size_t raw_ahead = 3;
        std::deque<RawMulti::Win> enq;  // enqueued on this engine (or the end marker), not launched
        RawMulti::Win held;             // popped, waiting for its turn to enqueue (windows enqueue in id order)
        bool have_held = false;
        bool input_done = false;
        bool engine_raw = false;
        // Every wait of this thread polls its own packs in flight meanwhile: a pack that is done but
        // not polled holds its staging window and its pack, and the formatter takes packs in input
        // order, so an engine that waited without polling (for a window, its enqueue turn, its launch
        // turn or a spare pack) could hold exactly what the others wait for.
        const auto tick = std::chrono::microseconds(300);
        auto poll_done = [&] {
            while (!inflight.empty() && complete_oldest(false)) {
            }
        };
        auto wait_polling = [&](std::unique_lock<std::mutex>& lk, auto pred) {
            while (!pred()) {
                if (inflight.empty()) {
                    R.cv.wait(lk, pred);
                    return;
                }
                // (system_clock: pthread_cond_timedwait, which ThreadSanitizer intercepts; a steady-clock
                // wait goes through pthread_cond_clockwait, which the toolchain's libtsan does not)
                if (R.cv.wait_until(lk, std::chrono::system_clock::now() + tick, pred)) return;
                lk.unlock();
                poll_done();
                lk.lock();
            }
        };
        auto drop_all = [&] {  // windows not launched: their copies finish, then the stages return
            (void)fq_engine_sync(e);
            if (engine_raw) (void)fq_engine_raw_end(e);
            engine_raw = false;
            for (const RawMulti::Win& w : enq)
                if (w.stage >= 0) R.free_stages.push(w.stage);
            enq.clear();
            if (have_held && held.stage >= 0) R.free_stages.push(held.stage);
            have_held = false;
            RawMulti::Win w;
            while (R.wq[(size_t)g]->pop(w))
                if (w.stage >= 0) R.free_stages.push(w.stage);
        };
        try {
            if (fq_engine_raw_begin(e, R.wcap, (uint64_t)16 << 20) != FQ_OK)
                throw std::runtime_error(std::string("fq_engine_raw_begin: ") + fq_engine_last_error(e));
            engine_raw = true;
            for (;;) {
                bool stop_now = false;
                while (enq.size() < raw_ahead && !input_done) {
                    // (wait for a window only when none is enqueued: the front one may be due)
                    if (!have_held) {
                        int got = R.wq[(size_t)g]->try_pop(held);
                        while (got == 0 && enq.empty()) {
                            got = R.wq[(size_t)g]->pop_for(held, tick);
                            if (got == 0) poll_done();
                        }
                        if (got == 0) break;
                        if (got < 0) {
                            input_done = true;
                            break;
                        }
                        have_held = true;
                    }
                    if (!held.end) {  // its turn: the window before it has been enqueued (on any engine)
                        std::unique_lock<std::mutex> lk(R.m);
                        if (enq.empty()) wait_polling(lk, [&] { return R.stopped || R.next_enqueue == held.id; });
                        if (R.stopped) {
                            stop_now = true;
                            break;
                        }
                        if (R.next_enqueue != held.id) break;  // (launch the front window first)
                    }
                    const RawMulti::Win w = held;
                    have_held = false;
                    if (!w.end) {
                        fq_raw_window rw{};
                        for (int m = 0; m < R.mates; ++m) {
                            rw.bytes[m] = R.stages[(size_t)w.stage]->buf[m].data();
                            rw.n[m] = w.n[m];
                        }
                        const auto q0 = std::chrono::steady_clock::now();
                        const int qrc = fq_engine_raw_enqueue(e, &rw);
                        raw_enqueue_s += since(q0);
                        if (qrc != FQ_OK) {
                            R.free_stages.push(w.stage);
                            throw std::runtime_error(std::string("fq_engine_raw_enqueue: ") + fq_engine_last_error(e));
                        }
                        std::lock_guard<std::mutex> lk(R.m);
                        R.next_enqueue = w.id + 1;
                        R.cv.notify_all();
                    } else {
                        input_done = true;
                    }
                    enq.push_back(w);
                }
                if (stop_now || enq.empty()) break;
                const RawMulti::Win w = enq.front();
                // Before the turn, on this engine's own time: its window's index (fq_engine_raw_wait)
                // and a spare pack if one is free.  The turn then only decides the window (the
                // earlier ones are decided: launch it, or end the stream in it) and passes on; the
                // launch follows outside it.  (A pack is waited for in the turn only: the earliest
                // window always gets the next pack back, so the packs in flight cannot all sit with
                // later windows.)
                std::unique_ptr<Pack> pk;
                fq_raw_result r{};
                if (!w.end) {
                    const auto x0 = std::chrono::steady_clock::now();
                    if (fq_engine_raw_wait(e, &r) != FQ_OK)
                        throw std::runtime_error(std::string("fq_engine_raw_wait: ") + fq_engine_last_error(e));
                    raw_idx_wait_s += since(x0);
                    // the window's index is back, so its copy to the device is done: the staging
                    // window goes back to the reader now, not when the pack completes (the device
                    // works from its own copy; the carry moves on the device)
                    if (w.stage >= 0) R.free_stages.push(w.stage);
                    enq.front().stage = -1;
                    if (spare.try_pop_recent(pk) < 0) throw Stopped();
                }
                auto give_back = [&] {
                    if (pk) spare.push(std::move(pk));
                };
                {
                    const auto t0w = std::chrono::steady_clock::now();
                    std::unique_lock<std::mutex> lk(R.m);
                    wait_polling(lk, [&] { return R.stopped || R.next_launch == w.id; });
                    raw_turn_wait_s += since(t0w);
                    if (R.stopped) {
                        give_back();
                        break;
                    }
                    if (w.end) {  // the input ends (or no whole pair fits): the host reader goes on
                        RawResumeInfo rr;
                        rr.done = true;
                        for (int m = 0; m < R.mates; ++m) {
                            rr.off[m] = w.start[m];
                            rr.done = rr.done && w.start[m] == R.size[m];
                        }
                        rr.next_seq = w.id;
                        R.end_locked(rr, rr.done ? "end of input" : "no whole pair fits a window");
                        enq.pop_front();
                        break;
                    }
                    if (!pk) {  // (the turn stays ours while the lock is released)
                        lk.unlock();
                        const auto p0 = std::chrono::steady_clock::now();
                        int got;
                        while ((got = spare.pop_for(pk, tick, true)) == 0) poll_done();
                        raw_pack_wait_s += since(p0);
                        lk.lock();
                        if (got < 0) throw Stopped();
                        if (R.stopped) {  // (an error elsewhere)
                            give_back();
                            break;
                        }
                    }
                    if (r.pairs != w.pairs || r.stop) {  // the GPU path stops inside this window
                        RawResumeInfo rr;
                        for (int m = 0; m < R.mates; ++m) rr.off[m] = w.start[m] + w.n[m] - r.carry[m];
                        rr.next_seq = w.id + 1;
                        R.end_locked(rr, std::string(r.stop ? "irregular record" : "short window") + " in window " +
                                             std::to_string(w.id) + " (" + std::to_string(r.pairs) + " of " +
                                             std::to_string(w.pairs) + " pairs)");
                    }
                    R.next_launch = w.id + 1;
                    R.cv.notify_all();
                }
                enq.pop_front();
                pk->clear();
                pk->raw = true;
                pk->text_mode = true;
                pk->paired = R.mates == 2;
                pk->seq_no = w.id;
                pk->stage = -1;  // (released after fq_engine_raw_wait)
                for (int m = 0; m < 2; ++m) {  // (output text, then the adapter entries)
                    size_t cap = m < R.mates ? (size_t)(w.n[m] + 4 * (uint64_t)target + 64) : 0;
                    if (merge && m == 0)  // (-m: the merged stream of both mates' text)
                        cap = (size_t)(w.n[0] + w.n[1] + 28 * (uint64_t)target + 64);
                    pk->out_text[m].reserve(cap + cap / 8);  // (headroom: see run_raw)
                    pk->out_text[m].resize_uninit(cap);
                    pk->rout.text.text[m] = m < R.mates ? pk->out_text[m].data() : nullptr;
                }
                const auto e0 = std::chrono::steady_clock::now();
                if (fq_engine_raw_launch(e, &r, &pk->rout, w.id) != FQ_OK) {  // (r as fq_engine_raw_wait gave it)
                    throw std::runtime_error(std::string("fq_engine_raw_launch: ") + fq_engine_last_error(e));
                }
                submit_s += since(e0);
                if (first_submit < 0) first_submit = since(t_start);
                pk->n = r.pairs;
                pk->max_cycles = max_cycles;
                R.pairs += (uint64_t)r.pairs;
                ++R.packs;
                while (!inflight.empty() && complete_oldest(false)) {
                }
                if ((int)inflight.size() >= raw_depth) complete_oldest();
                inflight.push_back(std::move(pk));
            }
            while (!inflight.empty()) complete_oldest();
            drop_all();
        } catch (...) {
            R.fail(std::current_exception());
            inflight.clear();
            drop_all();
            throw;
        }
        multi = nullptr;
    }

    // the dispatcher: planes (or the text index) of each pack, submit, completions in order
    void run(const Options& o, bool text_mode, Pool& pool, HostAcc& acc, std::mutex& acc_m) {
        try {
            std::unique_ptr<Pack> pk;
            while (in.pop(pk)) {
                const auto p0 = std::chrono::steady_clock::now();
                const bool as_text = text_mode && pack_text(*pk, &pool, o.merge);
                if (!as_text) {
                    pack_tiles(*pk, &pool);
                    prepare_pack(o, *pk, &pool);
                }
                tiles_s += since(p0);
                int max1 = 0, max2 = 0;
                if (as_text) {
                    max1 = pk->max_len[0];
                    max2 = pk->max_len[1];
                } else {
                    for (uint16_t l : pk->len[0]) max1 = std::max(max1, (int)l);
                    if (pk->paired)
                        for (uint16_t l : pk->len[1]) max2 = std::max(max2, (int)l);
                }
                const int need = o.merge ? max1 + max2 : std::max(max1, max2);
                if (need > max_cycles || pk->stride > max_stride || pk->n > max_batch) {
                    while (!inflight.empty()) complete_oldest();
                    {  // keep what the old engine accumulated, then grow it
                        std::lock_guard<std::mutex> g(acc_m);
                        drain(acc);
                    }
                    make(o, std::max(max_cycles, round16(need)), std::max(max_batch, pk->n), std::max(max_stride, pk->stride));
                }
                if ((int)inflight.size() >= depth) complete_oldest();
                pk->max_cycles = max_cycles;  // (read by the formatter)
                submit(*pk, as_text);
                if (first_submit < 0) first_submit = since(t_start);
                inflight.push_back(std::move(pk));
            }
            while (!inflight.empty()) complete_oldest();
        } catch (...) {
            // the packs in flight own pinned buffers the engine may still be copying into
            (void)fq_engine_sync(e);
            inflight.clear();
            throw;
        }
    }
};

void log(const std::string& s) {
    std::time_t t = std::time(nullptr);
    char d[64];
    std::strftime(d, sizeof d, "[%Y-%m-%d %H:%M:%S] ", std::localtime(&t));
    std::cerr << d << s << std::endl;
}

}  // namespace

// PE adapter detection, Evaluator::evaluateAdapterSeq of both mates (src/main.cpp:139-143).  The
// two mates' detections run concurrently; their read errors are printed in the reference's order
// (read 1's first; read 2's only when read 1's detection succeeded).  An interleaved input has no
// read2 file: opening "" fails as in the reference.
struct Detection {
    std::string a1, a2;
    std::exception_ptr err;
    double seconds = 0;
};
Detection detect_pe_adapters(const Options& o) {
    const auto t0 = std::chrono::steady_clock::now();
    Detection d;
    std::string msg1, msg2;
    std::exception_ptr e1, e2;
    const int dev = o.device_list()[0];
    std::thread t([&] {
        try {
            d.a2 = detect_adapter(o.in2, o.tail1, &msg2, dev);
        } catch (...) {
            e2 = std::current_exception();
        }
    });
    try {
        d.a1 = detect_adapter(o.in1, o.tail1, &msg1, dev);
    } catch (...) {
        e1 = std::current_exception();
    }
    t.join();
    std::cerr << msg1;
    if (e1) {
        d.err = e1;
    } else {
        std::cerr << msg2;
        d.err = e2;
    }
    d.seconds = since(t0);
    return d;
}

Options prepare_options(int argc, char** argv, bool detect_adapters) {
    Options o = parse_cli(argc, argv);
    try {  // Options::validate failures end in error_exit (src/util.h), exit status 255
        o.update(argc, argv);
        o.validate();
    } catch (const CliError& e) {
        throw std::runtime_error(e.what());
    }
    // Evaluator pre-pass, src/main.cpp:126-143
    if (!o.in1.empty()) o.est_seq_len1 = evaluate_read_len(o.in1);
    if (!o.in2.empty()) o.est_seq_len2 = evaluate_read_len(o.in2);
    if (o.split_by_number) {  // evaluateReadNum + the split size, src/main.cpp:130-134
        o.est_reads_num = evaluate_read_num(o.in1);
        if (o.split_number == 0) throw std::runtime_error("--split_file_number must be given (non-zero) with -s");
        o.split_size = (size_t)std::max(o.est_reads_num / o.split_number, 1);
        log("total reds: " + std::to_string(o.est_reads_num) + " split size: " + std::to_string(o.split_size));
    }
    if (o.split() && o.paired() && o.out2.empty())  // the reference dereferences a null split writer
        throw std::runtime_error("split output of paired-end reads needs both -o and -O");
    if (detect_adapters && o.detect_pe_adapter) {
        Detection d = detect_pe_adapters(o);
        if (d.err) std::rethrow_exception(d.err);
        o.detected_adapter1 = d.a1;
        o.detected_adapter2 = d.a2;
    }
    return o;
}

int run_tool(int argc, char** argv, bool exit_when_done) {
    // (declared first, so destroyed last: the page-locked blocks this run outgrew are freed once its
    // engines are gone and no other in-process run is active)
    struct PinnedRun {
        PinnedRun() { pinned_run_begin(); }
        ~PinnedRun() { pinned_run_end(); }
    } pinned_run;
    Options o;
    const auto t0 = std::chrono::steady_clock::now();
    try {
        // (an interleaved input has no read2 file to detect on: the synchronous pre-pass fails
        // on it before anything is written, as in the reference)
        o = prepare_options(argc, argv, false);
        // Hardware queues beyond HIP's default four: each engine's copy-in, index, compute and
        // copy-out streams plus the concurrent adapter detection's stream get their own, so the
        // DMA copies of one direction (or of one engine) do not queue behind the others' work
        // (unless the caller chose a value; read when HIP initialises, before any engine exists)
        {
            const int per_gpu = std::max<int>(1, (int)o.device_list().size());
            setenv("GPU_MAX_HW_QUEUES", std::to_string(std::min(4 * per_gpu + 4, 24)).c_str(), 0);
        }
        if (o.detect_pe_adapter && o.in2.empty()) {
            Detection d = detect_pe_adapters(o);
            if (d.err) std::rethrow_exception(d.err);
            o.detected_adapter1 = d.a1;
            o.detected_adapter2 = d.a2;
        }
    } catch (const CliError& e) {  // App::exit + FailureMessage::simple (src/CLI.hpp)
        if (e.code == 0) std::cout << e.what() << std::endl;
        else std::cerr << e.what() << "\nRun with --help for more information." << std::endl;
        return e.code;
    } catch (const std::exception& e) {
        std::cerr << "ERROR: " << e.what() << std::endl;
        return 255;
    }
    const double prepass_s = since(t0);
    // The detected adapters only reach the reports (JSON Read{1,2}AdapterSequence, HTML): trimming
    // uses --adapter_of_read{1,2} only (src/peprocessor.cpp:319, src/filterresult.cpp:315), so
    // the detection runs concurrently with the pipeline and is joined before the reports.  The
    // pack reader's messages wait for its messages (set_reader_stderr_gate).
    // It starts once the engines exist (FQ_DETECT_EARLY=1: before them), so its k-mer device work
    // does not compete with HIP start-up and the engines' allocations.
    std::promise<void> det_done;
    std::future<Detection> det;
    bool det_started = false;  // (det_done is then set by the detection, even once det is joined)
    const bool det_on = o.detect_pe_adapter && !o.in2.empty();
    auto start_detection = [&] {
        det_started = true;
        det = std::async(std::launch::async, [&o, &det_done] {
            Detection d;
            try {
                d = detect_pe_adapters(o);
            } catch (...) {
                d.err = std::current_exception();
            }
            det_done.set_value();
            return d;
        });
    };
    const bool det_early = std::getenv("FQ_DETECT_EARLY") != nullptr;  // (profiling)
    if (det_on) {
        set_reader_stderr_gate(det_done.get_future().share());
        if (det_early) start_detection();
    }
    // FQ_TIMING=1: the time the pipeline's teardown (pinned packs, engines, pool, mappings) takes
    // after the summary line, on stderr once everything is destroyed
    struct TeardownClock {
        std::chrono::steady_clock::time_point t0, logged;
        bool on = false;
        ~TeardownClock() {
            if (on) std::cerr << "fqtool-amd timing: teardown " << since(logged) << " s, total " << since(t0) << " s" << std::endl;
        }
    } teardown{t0, t0, std::getenv("FQ_TIMING") != nullptr};
    try {
        const bool paired = o.paired();
        // (raw streams: packs of 128 Ki pairs keep six windows' copies queued in 48 MiB windows)
        const size_t pack_n = o.pack_pairs ? o.pack_pairs : std::max<size_t>(o.max_reads_in_pack, 131072);
        int est = std::max(o.est_seq_len1, paired ? o.est_seq_len2 : 0);
        const std::vector<int> devices = o.device_list();
        const int G = (int)devices.size();
        const int depth = G > 2 ? 2 : 3;  // packs in flight per engine (each holds a device slot)
        // -w host threads (the reference's worker count) pack tiles, format and compress
        Pool pool(std::max(0, o.threads - 1));
        // (before the outputs: their writer threads hand text packs back to it until they close)
        const int n_packs = G * (depth + 1) + 6;  // (a raw stream keeps 4 in flight)
        Queue<std::unique_ptr<Pack>> spare((size_t)n_packs);
        for (int i = 0; i < n_packs; ++i) spare.push(std::unique_ptr<Pack>(new Pack(true)));
        Sink outs(o, &pool);
        // reader thread -> one dispatcher thread per engine (pack g of every G: planes or text
        // index, submit, poll in submission order) -> formatter thread (takes pack k from engine
        // k mod G: records -> output text, in input order) -> writer threads.  Packs (pinned
        // planes and records) are recycled.  (src/peprocessor.cpp:99-247: producer, -w workers,
        // writer threads.)
        // GPU-side ingest and egress (fq_engine_submit_text): the engine builds the planes from
        // the FASTQ text and writes the output text, for the plain out1 (+ out2) case
        const char* tm_env = std::getenv("FQ_TEXT_MODE");
        // (-m: every pair's output goes to the merged stream, which the engine writes as well;
        // with --discard_unmerged the unmerged pairs go to out1 / out2 instead: host packs)
        const bool text_mode = !(tm_env && std::string(tm_env) == "0") && !o.correction && !o.umi &&
                               !o.index_filter && !o.split() && !o.phred64 && o.failed_out.empty() &&
                               o.unpaired1.empty() && o.unpaired2.empty() &&
                               (o.merge ? paired && !o.merge_out.empty() && !o.discard_unmerged
                                        : !o.out1.empty() && (!paired || !o.out2.empty()));
        // records-only raw packs to plain outputs go out as byte ranges of their windows (zero copy)
        const char* zc_env = std::getenv("FQ_RAW_ZC");  // (profiling: 0 formats every record)
        const bool zc_ok = outs.plain_pair_outputs() && !(zc_env && std::string(zc_env) == "0");
        std::vector<std::unique_ptr<Lane>> lanes;
        // (before the lanes go, on any exit: the writers finish with the windows and packs they hold)
        struct OutsCloser {
            Sink& s;
            ~OutsCloser() {
                try {
                    s.close();
                } catch (...) {
                }
            }
        } outs_closer{outs};
        const int cyc0 = std::max(16, round16(o.merge ? 2 * est : est)), stride0 = round16(std::max(est, 16));
        const char* raw_env = std::getenv("FQ_RAW_MODE");
        const bool gz_both = ends_with_gz(o.in1) && (!paired || ends_with_gz(o.in2));
        // single-stream gzip inputs for the raw stream: their inflaters start before the engines
        // are made (HIP start-up and the engines' allocations take ~0.1 s), not at the first window
        std::unique_ptr<ParGzSource> pre_gz[2];
        if (text_mode && !o.interleaved && !(raw_env && std::string(raw_env) == "0") && gz_both && G == 1) {
            const std::string files[2] = {o.in1, o.in2};
            for (int m = 0; m < (paired ? 2 : 1); ++m)
                if ((pre_gz[m] = ParGzSource::open(files[m], (size_t)1 << 20, gz_inflate_threads()))) pre_gz[m]->prefetch();
        }
        for (int g = 0; g < G; ++g) {
            lanes.emplace_back(new Lane(devices[(size_t)g], depth));
            lanes.back()->t_start = t0;
            lanes.back()->merge = o.merge && paired;
            lanes.back()->make(o, cyc0, (int)pack_n, stride0);
        }
        const double engines_ready_s = since(t0);
        if (det_on && !det_early) start_detection();
        std::exception_ptr reader_err, format_err;
        double parse_s = 0, spare_wait_s = 0;
        HostAcc acc(o.insert_size_max);
        std::mutex acc_m;  // engines re-created larger mid-run add their accumulators here
        auto stop_all = [&] {
            spare.close();
            for (auto& l : lanes) {
                l->in.close();
                l->out.close();
            }
        };
        // (owned here, not by the reader thread: packs in flight point into its file mappings)
        PackReader pr(o.in1, o.in2, o.interleaved, o.phred64);
        pr.defer_tiles = true;  // the dispatchers fill the planes while the reader parses on
        // GPU-side record indexing (fq_engine_raw_*) for plain files on one engine: the engine's
        // dispatcher drives the raw stream first; the host reader takes over only where it stops
        // (single-stream gzip inputs on one engine too: their streams come from the parallel
        // inflater -- RawMulti reads windows with pread, plain files only)
        const bool raw_mode = text_mode && !o.interleaved && !(raw_env && std::string(raw_env) == "0") &&
                              ((!ends_with_gz(o.in1) && (!paired || !ends_with_gz(o.in2)) && pr.mapped()) ||
                               (gz_both && G == 1 && pr.parallel_gz()));
        std::promise<Lane::RawResume> raw_p;
        std::shared_future<Lane::RawResume> raw_f = raw_p.get_future().share();
        if (raw_mode && G == 1)
            for (int m = 0; m < 2; ++m) lanes[0]->pre_gz[m] = std::move(pre_gz[m]);
        // several engines: one window source cutting whole pairs, dealt round-robin (RawMulti)
        std::unique_ptr<RawMulti> rm;
        std::thread rm_reader, rm_warmer;
        if (raw_mode && G > 1) {
            rm.reset(new RawMulti);
            RawMulti& R = *rm;
            R.G = G;
            R.mates = paired ? 2 : 1;
            const std::string files[2] = {o.in1, o.in2};
            bool ok = true;
            for (int m = 0; m < R.mates; ++m) {
                R.fd[m] = ::open(files[m].c_str(), O_RDONLY);
                struct stat st;
                ok = ok && R.fd[m] >= 0 && fstat(R.fd[m], &st) == 0 && S_ISREG(st.st_mode) && st.st_size > 0;
                if (ok) {
                    R.size[m] = (uint64_t)st.st_size;
                    (void)posix_fadvise(R.fd[m], 0, 0, POSIX_FADV_SEQUENTIAL);
                }
            }
            for (int g = 0; g < G; ++g) R.wq.emplace_back(new Queue<RawMulti::Win>(2));
            std::promise<Lane::RawResume>* pp = &raw_p;
            R.on_end = [pp](const RawResumeInfo& ri) {
                Lane::RawResume r;
                r.done = ri.done;
                r.off[0] = ri.off[0];
                r.off[1] = ri.off[1];
                r.next_seq = ri.next_seq;
                pp->set_value(r);
            };
            if (!ok) {  // (the host reader takes the whole input)
                for (auto& q : R.wq) q->close();
                std::lock_guard<std::mutex> g(R.m);
                RawResumeInfo ri;
                R.end_locked(ri, "inputs are not regular files");
            } else {
                // staging: per GPU the windows enqueued (3, until their index is back: the copy is
                // then done and the stage returns, Lane::run_raw_multi) and queued for it (2), plus a
                // few for the reader to run ahead; the first is handed out at once, the others
                // page-locked on a helper thread.  Engines sharing a GPU share its link, so beyond
                // the first engine of a GPU one more stage each (page-locked memory is paid again at
                // the exit, ~40 ms per GiB: 8 engines on one device ran the same pipeline with 14
                // stages as with 23, and left 0.04-0.05 s sooner, profiles/r06_host_feed_stages.txt)
                std::vector<int> devs(devices.begin(), devices.end());
                std::sort(devs.begin(), devs.end());
                const int P = (int)(std::unique(devs.begin(), devs.end()) - devs.begin());
                const int kStages = std::getenv("FQ_MULTI_STAGES") ? std::atoi(std::getenv("FQ_MULTI_STAGES")) : P * 5 + 4 + (G - P);
                for (int i = 0; i < kStages; ++i) R.stages.emplace_back(new RawStage);
                R.free_stages.push(0);
                rm_warmer = std::thread([&R, kStages] {
                    int i = 1;
                    try {
                        for (; i < kStages; ++i) {
                            for (int m = 0; m < R.mates; ++m) R.stages[(size_t)i]->buf[m].reserve((size_t)R.wcap);
                            if (!R.free_stages.push(i)) return;
                        }
                    } catch (...) {  // (no memory to reserve ahead: the rest grow when first used)
                        for (; i < kStages; ++i)
                            if (!R.free_stages.push(i)) return;
                    }
                });
                rm_reader = std::thread([&R, &lanes, &pool, pack_n] {
                    R.read_windows((int)pack_n, lanes[0]->max_batch, pool);
                });
            }
        }
        std::thread reader([&] {
            try {
                if (raw_mode) {  // wait for the raw stream's end; resume where it stopped
                    const Lane::RawResume rr = raw_f.get();
                    if (rr.done) {
                        for (auto& l : lanes) l->in.close();
                        return;
                    }
                    pr.seek(rr.off[0], rr.off[1], rr.next_seq);
                }
                std::unique_ptr<Pack> pk;
                for (;;) {
                    const auto w0 = std::chrono::steady_clock::now();
                    if (!spare.pop_recent(pk)) break;
                    spare_wait_s += since(w0);
                    if (!pr.next(*pk, pack_n, &pool)) break;
                    Lane& l = *lanes[(size_t)(pk->seq_no % (uint64_t)G)];
                    if (!l.in.push(std::move(pk))) break;
                }
                parse_s = pr.parse_s;
            } catch (...) {
                reader_err = std::current_exception();
            }
            for (auto& l : lanes) l->in.close();
        });
        for (size_t gi = 0; gi < lanes.size(); ++gi) {
            Lane* l = lanes[gi].get();
            l->t = std::thread([&, l, gi] {
                try {
                    if (raw_mode && rm) {
                        l->run_raw_multi(*rm, (int)gi, (int)pack_n, spare);
                    } else if (raw_mode) {
                        Lane::RawResume rr;
                        rr.done = true;
                        try {
                            const std::string files[2] = {o.in1, o.in2};
                            rr = l->run_raw(files, paired ? 2 : 1, (int)pack_n, est, spare, pool);
                        } catch (...) {
                            raw_p.set_value(rr);
                            throw;
                        }
                        raw_p.set_value(rr);
                    }
                    l->run(o, text_mode, pool, acc, acc_m);
                } catch (const Stopped&) {  // (the stage that failed reports)
                } catch (...) {
                    l->err = std::current_exception();
                    stop_all();
                }
                l->out.close();
            });
        }
        AdapterCounts ac;
        uint64_t reads = 0, recs_packs = 0, zc_packs = 0;
        double format_s = 0;
        std::thread formatter([&] {
            try {
                RawPrev raw_prev;  // (records-only raw packs: the window the next carry comes from)
                std::unique_ptr<Pack> pk;
                for (uint64_t k = 0; lanes[(size_t)(k % (uint64_t)G)]->out.pop(pk); ++k) {
                    const auto f0 = std::chrono::steady_clock::now();
                    if (pk->seq_no != k) throw std::runtime_error("packs reached the formatter out of order");
                    const fq_params p = o.to_params(pk->max_cycles);
                    if (pk->raw && pk->recs) {  // records-only egress: the text is formatted here
                        format_raw_recs(*pk, raw_prev, o.adapter_trimming, p, pool, ac, zc_ok);
                        format_s += since(f0);
                        ++recs_packs;
                        zc_packs += pk->zc;
                        reads += (uint64_t)pk->n * (paired ? 2 : 1);
                        Pack* raw = pk.release();
                        outs.consume_text(*raw, [raw, &spare] {
                            raw->hold.reset();  // (zc: the window goes back once the writers are through)
                            spare.push(std::unique_ptr<Pack>(raw));
                        });
                        continue;
                    }
                    if (pk->text_mode) {  // the engine wrote the output text
                        if (o.adapter_trimming) {
                            if (pk->raw)
                                for (int m = 0; m < (paired ? 2 : 1); ++m)
                                    ac.add_entries(m, pk->out_text[m].data() + pk->tout.bytes[m], pk->rout.adapter_bytes[m], p, &pool);
                            else
                                ac.add(*pk, pk->res.data(), p, &pool);
                        }
                        format_s += since(f0);
                        reads += (uint64_t)pk->n * (paired ? 2 : 1);
                        // the writers recycle the pack once its output text is written
                        Pack* raw = pk.release();
                        outs.consume_text(*raw, [raw, &spare] { spare.push(std::unique_ptr<Pack>(raw)); });
                        continue;
                    } else {
                        apply_corrections(o, *pk, pk->res.data(), &pool);
                        if (o.adapter_trimming) ac.add(*pk, pk->res.data(), p, &pool);
                        outs.consume(*pk, pk->res.data());
                    }
                    format_s += since(f0);
                    reads += (uint64_t)pk->n * (paired ? 2 : 1);
                    spare.push(std::move(pk));
                }
            } catch (...) {
                format_err = std::current_exception();
                stop_all();
            }
        });
        for (auto& l : lanes) l->t.join();
        formatter.join();
        reader.join();
        if (rm) {
            {
                std::lock_guard<std::mutex> g(rm->m);
                RawResumeInfo ri;
                ri.done = true;
                rm->end_locked(ri, "pipeline stopped");  // (no-op once ended; frees a waiting reader)
            }
            for (auto& q : rm->wq) q->close();
            if (rm_reader.joinable()) rm_reader.join();
            if (rm_warmer.joinable()) rm_warmer.join();
            if (rm->err) std::rethrow_exception(rm->err);
        }
        const double pipeline_done_s = since(t0);
        double tiles_s = 0, submit_s = 0, wait_s = 0;
        std::exception_ptr lane_err;
        for (auto& l : lanes) {
            tiles_s += l->tiles_s;
            submit_s += l->submit_s;
            wait_s += l->wait_s;
            if (l->err && !lane_err) lane_err = l->err;
        }
        if (format_err) std::rethrow_exception(format_err);
        if (lane_err) std::rethrow_exception(lane_err);
        if (reader_err) std::rethrow_exception(reader_err);
        for (auto& l : lanes) l->drain(acc);
        if (o.dup) {  // Duplicate::statAll over the merged tables, src/peprocessor.cpp:200-207
            for (size_t g = 1; g < lanes.size(); ++g)
                if (fq_dup_merge(lanes[0]->dup, lanes[g]->dup) != FQ_OK) throw std::runtime_error("fq_dup_merge failed");
            std::vector<uint64_t> hist((size_t)o.dup_hist_size), gcs((size_t)o.dup_hist_size);
            uint64_t tot[2] = {0, 0};
            if (fq_dup_stat(lanes[0]->dup, o.dup_hist_size, hist.data(), gcs.data(), tot) != FQ_OK)
                throw std::runtime_error("fq_dup_stat failed");
            acc.set_dup(hist, gcs, tot[0], tot[1]);
        }
        outs.close();
        double detect_s = 0;
        if (det.valid()) {
            Detection d = det.get();
            set_reader_stderr_gate(std::shared_future<void>());
            if (d.err) {  // the reference fails before creating any output (src/main.cpp:137-141)
                for (const std::string* f : {&o.out1, &o.out2, &o.unpaired1, &o.unpaired2, &o.failed_out, &o.merge_out})
                    if (!f->empty() && *f != "/dev/null" && *f != "-" && *f != "/dev/stdout") std::remove(f->c_str());
                std::rethrow_exception(d.err);
            }
            o.detected_adapter1 = d.a1;
            o.detected_adapter2 = d.a2;
            detect_s = d.seconds;
        }
        const Json rep = build_report(o, acc, ac);
        {
            std::ofstream js(o.json_file, std::ios::binary);
            js << rep.dump(4);
        }
        {  // HtmlReporter::report, src/peprocessor.cpp:214-217 (always written; -H names the file)
            std::ofstream hs(o.html_file, std::ios::binary);
            hs << build_html(o, acc, ac, html_time_now());
        }
        teardown.logged = std::chrono::steady_clock::now();
        auto sum_lanes = [&](double Lane::*f) {
            double t = 0;
            for (auto& l : lanes) t += (*l).*f;
            return t;
        };
        log("fqtool-amd: " + std::to_string(reads) + " reads on " + std::to_string(G) + " engine(s)" +
            (raw_mode && rm ? " (raw stream on " + std::to_string(G) + " engines: host-cut pair windows, GPU record indexing, "
                              "ingest/egress: " + std::to_string(rm->pairs.load()) + " pairs in " + std::to_string(rm->packs.load()) +
                              " packs, ended: " + rm->why + "; window reads " + std::to_string(rm->read_s) +
                              " s, reader waiting for a stage " + std::to_string(rm->stage_wait_s) + " s; engines waiting for their index " +
                              std::to_string(sum_lanes(&Lane::raw_idx_wait_s)) + " s, for their turn " +
                              std::to_string(sum_lanes(&Lane::raw_turn_wait_s)) + " s, for a pack " +
                              std::to_string(sum_lanes(&Lane::raw_pack_wait_s)) + " s)"
             : raw_mode ? " (raw stream: GPU record indexing, ingest/egress: " + std::to_string(lanes[0]->raw_pairs) + " pairs in " +
                            std::to_string(lanes[0]->raw_packs) + " packs, ended: " + lanes[0]->raw_end + "; window reads " +
                            std::to_string(lanes[0]->raw_read_s) + " s, reader waiting for a stage " +
                            std::to_string(lanes[0]->raw_stage_wait_s) + " s, dispatcher waiting for windows " +
                            std::to_string(lanes[0]->raw_ready_wait_s) + " s, for a pack " + std::to_string(lanes[0]->raw_pack_wait_s) +
                            " s, in enqueue " + std::to_string(lanes[0]->raw_enqueue_s) + " s" +
                            (recs_packs ? "; records-only egress: " + std::to_string(recs_packs) + " packs, " + std::to_string(zc_packs) +
                                              " as byte ranges of their windows" : std::string()) + ")"
                      : text_mode ? " (text packs: GPU ingest/egress)" : "") + ", wall " +
            std::to_string(since(t0)) + " s, engine submit " + std::to_string(submit_s) + " s, wait " + std::to_string(wait_s) + " s; pre-pass " +
            std::to_string(prepass_s) + " s, adapter detection (concurrent) " + std::to_string(detect_s) + " s, format " + std::to_string(format_s) + " s, parse " + std::to_string(parse_s) +
            " s, tiles " + std::to_string(tiles_s) + " s, reader waiting " + std::to_string(spare_wait_s) +
            " s, engines ready at " + std::to_string(engines_ready_s) + " s, first pack submitted at " +
            std::to_string(lanes[0]->first_submit) + " s, pipeline done at " +
            std::to_string(pipeline_done_s) +
            " s; JSON report " + o.json_file + ", HTML report " + o.html_file);
        if (std::getenv("FQ_TIMING_MONO")) {  // (profiling: steady-clock stamps, to time exec and exit from outside)
            auto mono = [](std::chrono::steady_clock::time_point t) {
                return std::to_string(std::chrono::duration<double>(t.time_since_epoch()).count());
            };
            extern std::atomic<uint64_t> g_pinned_regrows, g_pinned_bytes;
            log("fqtool-amd mono: t0 " + mono(t0) + " end " + mono(std::chrono::steady_clock::now()) + " pinned " +
                std::to_string(g_pinned_bytes.load() >> 20) + " MiB, regrown " + std::to_string(g_pinned_regrows.load()) + " times");
        }
        // Everything is written.  The process ends here: the teardown (page-locked packs and
        // windows, engines, the pool's threads) only returns memory the exit returns anyway, and
        // took 0.15-0.2 s of the command's wall time (FQ_TIMING=1 keeps it, and times it).
        if (exit_when_done && !teardown.on) {
            std::cout.flush();
            std::cerr.flush();
            std::fflush(nullptr);
            _exit(0);
        }
    } catch (const std::exception& e) {
        if (det.valid()) det.wait();  // the pre-pass's messages come first, as in the reference
        else if (det_on && !det_started) det_done.set_value();  // (it never started: release the reader's gate)
        std::cerr << "ERROR: " << e.what() << std::endl;
        return 255;
    }
    return 0;
}

}  // namespace fqhost
