// options.h -- command line and derived options of the host tool.
//
// Mirrors the reference's Options tree (src/options.h:15-386), its CLI (src/main.cpp:18-120,
// CLI11 1.7.1 semantics: bool flags reset to false at registration, range checks, needs /
// excludes), and Options::update / validate (src/options.cpp:24-71).  ORA and k-mer analysis
// (outside this build's scope) are parsed and rejected with a clear message instead of being
// silently ignored.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/fqengine.h"

namespace fqhost {

struct CliError : std::runtime_error {
    int code;
    CliError(const std::string& m, int c = 1) : std::runtime_error(m), code(c) {}
};

struct Options {
    // I/O
    std::string in1, in2, out1, out2, unpaired1, unpaired2, failed_out, json_file = "report.json",
        html_file = "report.html";
    bool merge = false, discard_unmerged = false, phred64 = false, interleaved = false;
    std::string merge_out;
    int compression = 3;
    // adapters
    bool adapter_trimming = false, detect_pe_adapter = false;
    std::string adapter1, adapter2;               // --adapter_of_read1/2
    std::string detected_adapter1, detected_adapter2;  // Evaluator::evaluateAdapterSeq
    // trimming
    int front1 = 0, tail1 = 0, front2 = 0, tail2 = 0, max_len1 = 0, max_len2 = 0;
    // polyG / polyX
    bool polyg = false, polyx = false;
    int polyg_min_len = 10, polyg_max_mismatch = 1, polyg_one_per = 10;
    std::string polyx_chars = "ATCGN";
    int polyx_min_len = 10, polyx_max_mismatch = 1, polyx_one_per = 10;
    // cutting
    bool cut_front = false, cut_tail = false, cut_right = false;
    int window_shared = 4, quality_shared = 20;
    int window_front = 4, window_tail = 4, window_right = 4;
    int quality_front = 20, quality_tail = 20, quality_right = 20;
    // filters
    bool qual_filter = false, length_filter = false, complexity_filter = false;
    int low_qual_limit = 20;  // -Q (raw; +33 applied in update())
    double low_qual_ratio = 0.15;
    int n_base_limit = 5;
    double avg_qual = 0.0;
    int min_len = 15, max_len = 0;
    double complexity_threshold = 0.3;
    // base correction (-c), UMI (-u), index filter, duplication (-d), split (-s / -S)
    bool correction = false;
    bool umi = false, umi_drop_comment = false, umi_not_trim = false;
    int umi_location = 0, umi_length = 0, umi_skip = 0;
    bool index_filter = false;
    std::string index1_file, index2_file;
    int index_threshold = 0;
    std::vector<std::string> blacklist1, blacklist2;  // Options::initIndexFilter
    bool dup = false;
    int dup_keylen = 12, dup_hist_size = 32;
    bool split_by_number = false, split_by_lines = false;
    int split_number = 0, digits = 4;
    size_t split_size = 0;
    int est_reads_num = 0;  // Evaluator::evaluateReadNum
    bool split() const { return split_by_number || split_by_lines; }
    // leading bases UmiProcessor::process trims from mate m (before clamping to the read length)
    int umi_front(int m) const {
        if (!umi || umi_not_trim) return 0;
        const bool r1 = umi_location == 3 || umi_location == 6, r2 = umi_location == 4 || umi_location == 6;
        return (m == 0 ? r1 : (r2 && paired())) ? umi_length + umi_skip : 0;
    }
    // overlap
    int overlap_require = 30, overlap_diff_limit = 5;
    int insert_size_max = 512;
    // system
    int threads = 4;
    size_t max_packs_in_repo = 1000, max_reads_in_pack = 100000, max_packs_in_mem = 5;
    // derived (Options::update)
    int low_qual_base_limit = 40;
    int est_seq_len1 = 151, est_seq_len2 = 151;
    std::string command, cwd, version = "0.0.0";
    // engine devices: --device, or the --devices list (one engine per entry; packs are dealt
    // round-robin over them; an id may repeat)
    int device = 0;
    std::string devices;
    size_t pack_pairs = 0;  // 0: max(max_reads_in_pack, 262144)
    std::vector<int> device_list() const;

    bool paired() const { return !in2.empty() || interleaved; }
    // Options::update (src/options.cpp:24-58) minus the parts that need the evaluator
    void update(int argc, char** argv);
    // Options::validate (src/options.cpp:60-71)
    void validate() const;
    // POD snapshot for the engine (include/fqengine.h), max_cycles sized by the caller
    fq_params to_params(int max_cycles) const;
};

// Parses argv like the reference's CLI11 setup; throws CliError (help text included for -h).
Options parse_cli(int argc, char** argv);
std::string help_text(const char* prog);

}  // namespace fqhost
