// report.h -- accumulators -> the reference's JSON report.
//
// HostAcc keeps the engine's flat accumulator (include/fqengine.h layout) with a growable cycle
// count so packs with longer reads can be absorbed by re-creating the engine.  build_report
// restates Stats::summarize / reportJson (src/stats.cpp:147-228, :392-430),
// FilterResult::reportJson* (src/filterresult.cpp:204-397) and JsonReporter::report
// (src/jsonreporter.cpp:23-162).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/fqengine.h"
#include "json.h"
#include "options.h"

namespace fqhost {

struct Pack;

class HostAcc {
   public:
    explicit HostAcc(int insert_size_max = 512);
    // add an engine accumulator block of the given max_cycles
    void add(const uint64_t* acc, int max_cycles);
    // raw add of one counter (tests)
    const std::vector<uint64_t>& head() const { return head_; }
    int cycles_capacity() const { return cap_; }
    uint64_t filter(int code) const { return head_[FQ_ACC_FILTER + code]; }
    uint64_t stat(int k, int field) const { return st_[k][field]; }
    uint64_t cyc(int k, int c, int slot) const { return (size_t)c < cyc_[k].size() / 16 ? cyc_[k][(size_t)c * 16 + slot] : 0; }
    int insert_size_max() const { return ism_; }
    uint64_t tail(int k) const { return tail_[k]; }  // FQ_ACC_TAIL_*
    // duplication analysis result (Duplicate::statAll: bins, GC sums, reads counted, duplicates)
    void set_dup(const std::vector<uint64_t>& hist, const std::vector<uint64_t>& gc_sum, uint64_t total, uint64_t dups) {
        dup_hist = hist;
        dup_gc_sum = gc_sum;
        dup_total = total;
        dup_dups = dups;
    }
    std::vector<uint64_t> dup_hist, dup_gc_sum;
    uint64_t dup_total = 0, dup_dups = 0;

   private:
    int ism_;
    int cap_ = 0;
    std::vector<uint64_t> head_;   // everything before the stats blocks
    uint64_t st_[4][4] = {};       // reads, length_sum, q20, q30
    std::vector<uint64_t> cyc_[4];  // [cycle][16]
    uint64_t tail_[FQ_ACC_TAIL_WORDS] = {};
};

// FilterResult's adapter-string counts (src/filterresult.cpp:138-177).  Every trimmed tail's text
// is sliced from the pack and counted exactly, keyed by its bytes, in a table split into shards by
// hash: a pack's ranges are hashed on the pool, then each shard takes its entries of every range
// (no serial merge).  The reports only print the strings holding >= 1 % of a mate's total, plus
// "Others" (src/filterresult.cpp:231-251); report() returns those, in the map order the
// reference prints, with the total.
class Pool;
class AdapterCounts {
   public:
    static constexpr int kShards = 64;
    AdapterCounts();
    ~AdapterCounts();
    AdapterCounts(const AdapterCounts&) = delete;
    AdapterCounts& operator=(const AdapterCounts&) = delete;
    void add(const Pack& pk, const fq_read_result* res, const fq_params& p, Pool* pool = nullptr);
    void add(int mate, const std::string& adapter, size_t count);  // one string (tests, report API)
    // a raw pack's trimmed-adapter entries of one mate (fq_raw_out, include/fqengine.h)
    void add_entries(int mate, const char* entries, size_t bytes, const fq_params& p, Pool* pool = nullptr);
    struct Report {
        std::map<std::string, size_t> top;  // the strings at >= 1 % of total (FilterResult's test)
        size_t total = 0;                   // adapter-trimmed reads of the mate
    };
    Report report(int mate) const;

   private:
    struct Shard;
    std::vector<std::unique_ptr<Shard>> shards_[2];
};

// Stats::summarize + reportJson for accumulator stats block k (src/stats.cpp:147-228, :392-430)
struct Summary {
    uint64_t reads = 0, bases = 0, q20 = 0, q30 = 0, gc = 0, length_sum = 0;
    int cycles = 0;
    uint64_t base_contents[8] = {};           // mBaseContents
    std::vector<double> qual_curves[5];       // A, T, C, G, Mean
    std::vector<double> content_curves[6];    // A, T, C, G, N, GC
    Json json;
    int mean_length() const { return reads ? (int)(length_sum / reads) : 0; }
};
Summary summarize(const HostAcc& a, int k);

Json build_report(const Options& o, const HostAcc& acc, const AdapterCounts& ac);

// HtmlReporter::report (src/htmlreporter.cpp:23-95): the whole HTML page; `now` is the footer's
// time stamp (htmlutil::getCurrentSystemTime)
std::string build_html(const Options& o, const HostAcc& acc, const AdapterCounts& ac, const std::string& now);
std::string html_time_now();

}  // namespace fqhost
