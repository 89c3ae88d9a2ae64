// options.cpp -- see options.h.  Flag table follows reference src/main.cpp:18-120.
#include "options.h"

#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <set>
#include <sys/stat.h>

namespace fqhost {
namespace {

enum class Kind { Flag, Int, SizeT, Double, Str };

struct Spec {
    std::vector<std::string> names;  // "-i", "--adapter_of_read1", ...
    Kind kind = Kind::Flag;
    void* target = nullptr;
    double lo = -1e300, hi = 1e300;  // CLI::Range
    bool existing_file = false;
    bool required = false;
    std::vector<std::string> needs, excludes;
    std::string help;
    bool unsupported = false;  // parsed, then rejected (outside the hot-path scope)
};

bool is_file(const std::string& p) {
    struct stat st;
    return stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

struct Table {
    std::vector<Spec> specs;
    std::map<std::string, size_t> by_name;
    bool dummy_bool = false;
    int dummy_int = 0;
    size_t dummy_size = 0;
    double dummy_double = 0;
    std::string dummy_str;

    Spec& add(std::vector<std::string> names, Kind k, void* t, const std::string& help) {
        Spec sp;
        sp.names = names;
        sp.kind = k;
        sp.target = t;
        specs.push_back(sp);
        specs.back().help = help;
        for (auto& n : names) by_name[n] = specs.size() - 1;
        return specs.back();
    }
};

Table make_table(Options& o) {
    Table t;
    // the Spec vector must not reallocate while we hold references
    t.specs.reserve(128);
    auto range = [](Spec& s, double lo, double hi) -> Spec& {
        s.lo = lo;
        s.hi = hi;
        return s;
    };
    // ---- IO
    Spec& in1 = t.add({"-i"}, Kind::Str, &o.in1, "read1 input file name");
    in1.required = true;
    in1.existing_file = true;
    t.add({"-o"}, Kind::Str, &o.out1, "read1 output file name").required = true;
    Spec& in2 = t.add({"-I"}, Kind::Str, &o.in2, "read2 input file name");
    in2.needs = {"-i"};
    in2.existing_file = true;
    t.add({"-O"}, Kind::Str, &o.out2, "read2 output file name").needs = {"-I"};
    t.add({"--unpaired_read1"}, Kind::Str, &o.unpaired1, "output read1 whose mate failed QC");
    t.add({"--unpaired_read2"}, Kind::Str, &o.unpaired2, "output read2 whose mate failed QC");
    t.add({"--failed_out"}, Kind::Str, &o.failed_out, "output failed QC reads");
    t.add({"-m"}, Kind::Flag, &o.merge, "merge overlapped readpair").needs = {"-I"};
    t.add({"--discard_unmerged"}, Kind::Flag, &o.discard_unmerged, "discard unmerged reads").needs = {"-m"};
    t.add({"--merge_output"}, Kind::Str, &o.merge_out, "merged output").needs = {"-m"};
    t.add({"--phred64"}, Kind::Flag, &o.phred64, "input fastq is phred64");
    range(t.add({"-z"}, Kind::Int, &o.compression, "gzip output compress level"), 1, 9);
    t.add({"--in_fq_interleaved"}, Kind::Flag, &o.interleaved, "input fastq interleaved").excludes = {"-I"};
    // ---- duplication
    t.add({"-d"}, Kind::Flag, &o.dup, "enable duplication analysis");
    Spec& dk = range(t.add({"--dup_ana_key_len"}, Kind::Int, &o.dup_keylen, "duplication analysis key length"), 12, 31);
    dk.needs = {"-d"};
    Spec& dh = range(t.add({"--dup_ana_hist_size"}, Kind::Int, &o.dup_hist_size, "duplicate analysis hist size"), 1, 10000);
    dh.needs = {"-d"};
    // ---- adapter
    t.add({"-a"}, Kind::Flag, &o.adapter_trimming, "enable adapter trimming");
    t.add({"--adapter_of_read1"}, Kind::Str, &o.adapter1, "adapter of read1").needs = {"-a"};
    t.add({"--adapter_of_read2"}, Kind::Str, &o.adapter2, "adapter of read2").needs = {"-a"};
    t.add({"--detect_pe_adapter"}, Kind::Flag, &o.detect_pe_adapter, "detect PE adapters").needs = {"-I"};
    // ---- trimming
    range(t.add({"-f"}, Kind::Int, &o.front1, "bases trimmed in read1 front"), 0, 1000);
    range(t.add({"-t"}, Kind::Int, &o.tail1, "bases trimmed in read1 tail"), 0, 1000);
    range(t.add({"-b"}, Kind::Int, &o.max_len1, "read1 max length allowed"), 0, 1000);
    range(t.add({"-F"}, Kind::Int, &o.front2, "bases trimmed in read2 front"), 0, 1000);
    range(t.add({"-T"}, Kind::Int, &o.tail2, "#bases trimmed in read2 tail"), 0, 1000);
    range(t.add({"-B"}, Kind::Int, &o.max_len2, "read2 max length allowed"), 0, 1000);
    // ---- polyG / polyX
    t.add({"-g"}, Kind::Flag, &o.polyg, "enable polyG trim");
    t.add({"--min_len_detect_polyG"}, Kind::Int, &o.polyg_min_len, "minimum length to detect polyG").needs = {"-g"};
    t.add({"--max_mismatches_polyG"}, Kind::Int, &o.polyg_max_mismatch, "maximum mismatches allowed for matched polyG")
        .needs = {"-g"};
    t.add({"--one_mismatch_each_polyG"}, Kind::Int, &o.polyg_one_per,
          "allowed one mismatch every bases for matched polyG")
        .needs = {"-g"};
    t.add({"-x"}, Kind::Flag, &o.polyx, "enable polyX trim");
    t.add({"--base_to_trim"}, Kind::Str, &o.polyx_chars, "nucleotides to trim").needs = {"-x"};
    t.add({"--min_len_detect_polyX"}, Kind::Int, &o.polyx_min_len, "minimum length to detect polyX").needs = {"-x"};
    t.add({"--max_mismatches_polyX"}, Kind::Int, &o.polyx_max_mismatch, "maximum mismatches allowed for matched polyX")
        .needs = {"-x"};
    t.add({"--one_mismatch_each_polyX"}, Kind::Int, &o.polyx_one_per,
          "allowed one mismatch every bases for matched polyX")
        .needs = {"-x"};
    // ---- cutting by quality (-W / -M set the *shared* values only; src/options.h:118-130
    //      copies them into the per-direction fields at construction, so they have no effect)
    t.add({"--enable_cut_front"}, Kind::Flag, &o.cut_front, "slide and drop from 5'->3'");
    t.add({"--enable_cut_tail"}, Kind::Flag, &o.cut_tail, "slide and drop from 3'->5'");
    t.add({"--enable_cut_right"}, Kind::Flag, &o.cut_right, "slide from 5'->3' and drop window and right part");
    range(t.add({"-W"}, Kind::Int, &o.window_shared, "window size for cut sliding"), 0, 1000);
    range(t.add({"-M"}, Kind::Int, &o.quality_shared, "min mean quality to drop window/bases"), 1, 36);
    range(t.add({"--cut_front_window"}, Kind::Int, &o.window_front, "window size to cut from 5''"), 0, 1000).needs = {
        "--enable_cut_front"};
    range(t.add({"--cut_tail_window"}, Kind::Int, &o.window_tail, "window size to cut from 3'"), 0, 1000).needs = {
        "--enable_cut_tail"};
    range(t.add({"--cut_right_window"}, Kind::Int, &o.window_right, "window size to cut right"), 0, 1000).needs = {
        "--enable_cut_right"};
    range(t.add({"--cut_front_mean_qual"}, Kind::Int, &o.quality_front, "mean quality to cut from 5'"), 1, 36).needs = {
        "--enable_cut_front"};
    range(t.add({"--cut_tail_mean_qual"}, Kind::Int, &o.quality_tail, "mean quality to cut from 3'"), 1, 36).needs = {
        "--enable_cut_tail"};
    // the reference ties --cut_right_mean_qual to --enable_cut_tail (src/main.cpp:66)
    range(t.add({"--cut_right_mean_qual"}, Kind::Int, &o.quality_right, "mean quality to cut right"), 1, 36).needs = {
        "--enable_cut_tail"};
    // ---- quality filtering
    t.add({"-q"}, Kind::Flag, &o.qual_filter, "enable quality filter");
    range(t.add({"-Q"}, Kind::Int, &o.low_qual_limit, "minimum quality for qualified bases"), 0, 60).needs = {"-q"};
    range(t.add({"-U"}, Kind::Double, &o.low_qual_ratio, "maximum low quality ratio allowed in one read"), 0, 1).needs = {
        "-q"};
    t.add({"-N"}, Kind::Int, &o.n_base_limit, "maximum N bases allowed in one read").needs = {"-q"};
    t.add({"-e"}, Kind::Double, &o.avg_qual, "average quality needed for one read").needs = {"-q"};
    // ---- length filtering
    t.add({"-l"}, Kind::Flag, &o.length_filter, "enable length filter");
    range(t.add({"--min_length"}, Kind::Int, &o.min_len, "min length required for a read"), 0, 1000).needs = {"-l"};
    range(t.add({"--max_length"}, Kind::Int, &o.max_len, "max length allowed for a read"), 0, 1000).needs = {"-l"};
    // ---- low complexity
    t.add({"-y"}, Kind::Flag, &o.complexity_filter, "enable low complexity filter");
    range(t.add({"-Y"}, Kind::Double, &o.complexity_threshold, "min complexity required for a read"), 0, 1).needs = {
        "-y"};
    // ---- index filtering
    t.add({"--enable_index_filter"}, Kind::Flag, &o.index_filter, "enable index filtering");
    Spec& i1 = t.add({"--index1_file"}, Kind::Str, &o.index1_file, "index1 file to filter");
    i1.existing_file = true;
    i1.needs = {"--enable_index_filter"};
    Spec& i2 = t.add({"--index2_file"}, Kind::Str, &o.index2_file, "index2 file to filetr");
    i2.existing_file = true;
    i2.needs = {"--enable_index_filter"};
    range(t.add({"--max_diff_for_match"}, Kind::Int, &o.index_threshold, "max ed to validate index matcha"), 0, 10).needs = {
        "--enable_index_filter"};
    // ---- base correction + overlap parameters
    t.add({"-c"}, Kind::Flag, &o.correction, "enable base correction in PE reads");
    range(t.add({"--min_overlap_len"}, Kind::Int, &o.overlap_require, "min overlap length needed for overlap analysis"),
          0, 1000);
    range(t.add({"--max_diff_for_overlap"}, Kind::Int, &o.overlap_diff_limit, "max ed to validate overlap"), 0, 10);
    // ---- UMI
    t.add({"-u"}, Kind::Flag, &o.umi, "enable UMI preprocess");
    range(t.add({"--umi_location"}, Kind::Int, &o.umi_location, "0[none]1[index1]2[index2]3[read1]4[read2]5[perindex]6[perread]"),
          1, 6)
        .needs = {"-u"};
    range(t.add({"--umi_length"}, Kind::Int, &o.umi_length, "umi length"), 0, 1000).needs = {"-u"};
    range(t.add({"--umi_skip_length"}, Kind::Int, &o.umi_skip, "bases to skip after umi"), 0, 1000).needs = {"-u"};
    t.add({"--umi_drop_comment"}, Kind::Flag, &o.umi_drop_comment, "drop other comment information").needs = {"-u"};
    t.add({"--umi_not_trim"}, Kind::Flag, &o.umi_not_trim, "do not trim reads").needs = {"-u"};
    // ---- ORA / k-mer (outside scope)
    t.add({"--ora"}, Kind::Flag, &t.dummy_bool, "enable ORA").unsupported = true;
    range(t.add({"--ora_sample"}, Kind::Int, &t.dummy_int, "ORA sampling steps"), 1, 10000).needs = {"--ora"};
    t.add({"--kmer"}, Kind::Flag, &t.dummy_bool, "enable kmer analysis").unsupported = true;
    range(t.add({"--kmer_length"}, Kind::Int, &t.dummy_int, "kmer length to analysis"), 4, 16).needs = {"--kmer"};
    // ---- reporting / system
    t.add({"-J"}, Kind::Str, &o.json_file, "json format report file");
    t.add({"-H"}, Kind::Str, &o.html_file, "html format report file");
    range(t.add({"-w"}, Kind::Int, &o.threads, "worker thread number"), 1, 16);
    // ---- split (--digits_file_name sets Options::digits, which the split writers never read:
    //      they use SplitOptions::digits = 4, src/threadconfig.cpp:91-96)
    Spec& sfn = t.add({"-s"}, Kind::Flag, &o.split_by_number, "split output by file number");
    sfn.excludes = {"-m"};
    t.add({"--split_file_number"}, Kind::Int, &o.split_number, "total split output file number").needs = {"-s"};
    Spec& sln = t.add({"-S"}, Kind::Flag, &o.split_by_lines, "max line of each output file");
    sln.excludes = {"-s", "-m"};
    t.add({"--splie_file_line"}, Kind::SizeT, &o.split_size, "split output file line limit").needs = {"-S"};
    range(t.add({"--digits_file_name"}, Kind::Int, &o.digits, "digits for sequential output filename"), 1, 10);
    range(t.add({"--max_packs_in_repo"}, Kind::SizeT, &o.max_packs_in_repo, "max packs in repo"), 1, 1000000);
    range(t.add({"--max_item_in_pack"}, Kind::SizeT, &o.max_reads_in_pack, "max read/pairs in pack"), 1, 1000000);
    range(t.add({"--max_packs_in_mem"}, Kind::SizeT, &o.max_packs_in_mem, "max packs in memory"), 1, 1000000);
    // ---- engine
    t.add({"--device"}, Kind::Int, &o.device, "[fqtool-amd] HIP device of the engine (default 0)");
    range(t.add({"--pack_pairs"}, Kind::SizeT, &o.pack_pairs,
                "[fqtool-amd] reads/pairs per engine pack (default max(--max_item_in_pack, 262144))"),
          1, 16777216);
    t.add({"--devices"}, Kind::Str, &o.devices,
          "[fqtool-amd] comma-separated HIP devices the packs are dealt over, e.g. 0,1,2,3 (default: --device)");
    return t;
}

// CLI11 1.7 detail::lexical_cast (src/CLI.hpp): full-match stoll / stoull / stold
bool cast_signed(const std::string& v, long long& out) {
    try {
        size_t n = 0;
        out = std::stoll(v, &n, 0);
        return n == v.size();
    } catch (...) {
        return false;
    }
}

bool cast_unsigned(const std::string& v, unsigned long long& out) {
    if (!v.empty() && v.front() == '-') return false;
    try {
        size_t n = 0;
        out = std::stoull(v, &n, 0);
        return n == v.size();
    } catch (...) {
        return false;
    }
}

bool cast_double(const std::string& v, double& out) {
    try {
        size_t n = 0;
        out = (double)std::stold(v, &n);
        return n == v.size();
    } catch (...) {
        return false;
    }
}

bool has_range(const Spec& s) { return s.lo > -1e299; }

// Option::get_type_name as the help text shows it
std::string type_name(const Spec& s) {
    if (s.existing_file) return "FILE";
    if (has_range(s))  // CLI::Range(int, int): the validator type is int for every ranged option
        return "INT in [" + std::to_string((long long)s.lo) + " - " + std::to_string((long long)s.hi) + "]";
    switch (s.kind) {
        case Kind::Int: return "INT";
        case Kind::SizeT: return "UINT";
        case Kind::Double: return "FLOAT";
        default: return "TEXT";
    }
}

// Option::run_callback: validators first (ValidationError, 105), then the conversion
// (ConversionError, 104)
void run_callback(const Spec& s, const std::string& val) {
    const std::string& name = s.names[0];
    if (has_range(s)) {
        // CLI::Range's int lexical_cast: a value that is not an integer leaves the compared
        // variable unset; for the integer options we treat that as out of range (what the
        // reference binary prints), for -U / -Y (double options behind an int Range) as in range.
        long long v;
        const bool ok = cast_signed(val, v);
        if ((ok && (v < (long long)s.lo || v > (long long)s.hi)) || (!ok && s.kind != Kind::Double))
            throw CliError(name + ": Value " + val + " not in range " + std::to_string((long long)s.lo) + " to " +
                               std::to_string((long long)s.hi),
                           105);
    }
    if (s.existing_file && !is_file(val)) throw CliError(name + ": File does not exist: " + val, 105);
    const std::string conv = "Could not convert: " + name + " = " + val;
    switch (s.kind) {
        case Kind::Str:
            *static_cast<std::string*>(s.target) = val;
            break;
        case Kind::Int: {
            long long v;
            if (!cast_signed(val, v) || v < INT_MIN || v > INT_MAX) throw CliError(conv, 104);
            *static_cast<int*>(s.target) = (int)v;
            break;
        }
        case Kind::SizeT: {
            unsigned long long v;
            if (!cast_unsigned(val, v)) throw CliError(conv, 104);
            *static_cast<size_t*>(s.target) = (size_t)v;
            break;
        }
        case Kind::Double: {
            double v;
            if (!cast_double(val, v)) throw CliError(conv, 104);
            *static_cast<double*>(s.target) = v;
            break;
        }
        case Kind::Flag:
            *static_cast<bool*>(s.target) = true;
            break;
    }
}

}  // namespace

std::string help_text(const char* prog) {
    Options o;
    Table t = make_table(o);
    std::string h = std::string("program: ") + prog + "\nversion: " + o.version +
                    " (fqtool-amd: MI355X engine)\nUsage: " + prog + " [OPTIONS]\n\nOptions:\n";
    for (auto& s : t.specs) {
        std::string names;
        for (auto& n : s.names) names += (names.empty() ? "" : ",") + n;
        h += "  " + names + std::string(names.size() < 30 ? 30 - names.size() : 1, ' ') + s.help +
             (s.unsupported ? " [not supported by fqtool-amd]" : "") + "\n";
    }
    return h;
}

// App::parse as CLI11 1.7 runs it (src/CLI.hpp): arguments are collected in command-line
// order, then callbacks run in definition order, then --help, requirements and extras.
Options parse_cli(int argc, char** argv) {
    Options o;
    Table t = make_table(o);
    // CLI11 add_flag on a bool resets the default to false: our
    // defaults are already false for every flag.
    std::vector<std::vector<std::string>> results(t.specs.size());
    std::vector<int> count(t.specs.size(), 0);
    std::vector<std::string> extras;
    bool help = false;
    std::vector<std::string> args(argv + 1, argv + argc);
    for (size_t i = 0; i < args.size(); ++i) {
        const std::string a = args[i];
        if (a == "-h" || a == "--help") {
            help = true;
            continue;
        }
        std::string name, val;
        bool has_val = false;
        if (a.size() > 2 && a.compare(0, 2, "--") == 0) {
            const size_t eq = a.find('=');
            name = a.substr(0, eq);
            if (eq != std::string::npos) {
                val = a.substr(eq + 1);
                has_val = true;
            }
        } else if (a.size() >= 2 && a[0] == '-' && a[1] != '-') {
            name = a.substr(0, 2);
            if (a.size() > 2) {
                auto f = t.by_name.find(name);
                if (f != t.by_name.end() && t.specs[f->second].kind == Kind::Flag) {
                    args.insert(args.begin() + (long)i + 1, "-" + a.substr(2));  // -qag -> -q -ag
                } else {
                    val = a.substr(2);
                    has_val = true;
                }
            }
        } else {
            extras.push_back(a);
            continue;
        }
        auto it = t.by_name.find(name);
        if (it == t.by_name.end()) {
            extras.push_back(a);
            continue;
        }
        const size_t k = it->second;
        const Spec& s = t.specs[k];
        ++count[k];
        if (s.kind == Kind::Flag) continue;
        if (!has_val) {
            if (i + 1 >= args.size())  // ArgumentMismatch::TypedAtLeast
                throw CliError(name + ": 1 required " + type_name(s) + " missing", 114);
            val = args[++i];
        }
        results[k].push_back(val);
    }
    for (size_t k = 0; k < t.specs.size(); ++k) {
        if (!count[k]) continue;
        const Spec& s = t.specs[k];
        if (s.kind == Kind::Flag) run_callback(s, "");
        else run_callback(s, results[k].back());
    }
    if (help) throw CliError(help_text(argv[0]), 0);
    auto used = [&](const std::string& n) {
        auto f = t.by_name.find(n);
        return f != t.by_name.end() && count[f->second] > 0;
    };
    for (size_t k = 0; k < t.specs.size(); ++k) {
        const Spec& s = t.specs[k];
        if (s.required && !count[k]) throw CliError(s.names[0] + " is required", 106);
        if (!count[k]) continue;
        for (auto& n : s.needs)
            if (!used(n)) throw CliError(s.names[0] + " requires " + n, 107);
        // excludes are symmetric in CLI11
        for (auto& n : s.excludes)
            if (used(n)) throw CliError(s.names[0] + " excludes " + n, 108);
        for (size_t j = 0; j < t.specs.size(); ++j)
            for (auto& n : t.specs[j].excludes)
                if (n == s.names[0] && count[j]) throw CliError(s.names[0] + " excludes " + t.specs[j].names[0], 108);
    }
    if (!extras.empty()) {
        std::string m = extras.size() > 1 ? "The following arguments were not expected:"
                                          : "The following argument was not expected:";
        for (auto e = extras.rbegin(); e != extras.rend(); ++e) m += " " + *e;  // CLI11 reports them last-first
        throw CliError(m, 109);
    }
    for (size_t k = 0; k < t.specs.size(); ++k)
        if (count[k] && t.specs[k].unsupported)
            throw CliError("option " + t.specs[k].names[0] + " (" + t.specs[k].help +
                               ") is outside the hot path this MI355X build implements; see DESIGN.md",
                           2);
    return o;
}

namespace {

// Options::makeListFromFileByLine, src/options.cpp:92-104 (util::strip's result is discarded
// there, so lines are taken as they are)
std::vector<std::string> index_list(const std::string& file) {
    std::vector<std::string> out;
    std::ifstream in(file);
    std::string line;
    while (std::getline(in, line)) {
        if (line.find_first_not_of("ATCG") != std::string::npos)
            throw CliError("processing " + file + ", each line should be one index, which can only contain A/T/C/G", 255);
        out.push_back(line);
    }
    return out;
}

// util::validFile, src/util.h:311-318
void valid_file(const std::string& path) {
    struct stat st;
    if (stat(path.c_str(), &st) == 0 && S_ISDIR(st.st_mode)) throw CliError("this is not a file path!", 255);
    if (!is_file(path)) throw CliError("file does not exist", 255);
}

}  // namespace

void Options::update(int argc, char** argv) {
    // src/options.cpp:24-58
    low_qual_limit += 33;
    if (adapter_trimming && adapter1.empty() && adapter2.empty() && paired()) detect_pe_adapter = true;
    if (index_filter && !(index1_file.empty() && index2_file.empty())) {  // Options::initIndexFilter, :73-90
        if (!index1_file.empty()) {
            valid_file(index1_file);
            blacklist1 = index_list(index1_file);
        }
        if (!index2_file.empty()) {
            valid_file(index2_file);
            blacklist2 = index_list(index2_file);
        }
    }
    low_qual_base_limit = (int)(low_qual_ratio * est_seq_len1);  // est_seq_len1 is still 151 here
    if (umi && (umi_location == 3 || umi_location == 4 || umi_location == 6) && umi_length == 0)
        throw CliError("umi length can not be zero if it's in read1/2", 255);
    std::transform(polyx_chars.begin(), polyx_chars.end(), polyx_chars.begin(),
                   [](unsigned char c) { return (char)std::toupper(c); });
    command.clear();
    for (int i = 0; i < argc; ++i) {
        command += argv[i];
        command += " ";
    }
    char buf[4096];
    cwd = getcwd(buf, sizeof buf) ? std::string(buf) : std::string();
}

void Options::validate() const {
    // src/options.cpp:60-71
    if (merge && merge_out.empty()) throw CliError("merged file output must be provided!", 255);
    if (polyx_chars.find_first_not_of("ATCGN") != std::string::npos)
        throw CliError("Can only trim nucleotides ATCGN", 255);
    if ((int)adapter1.size() > FQ_MAX_ADAPTER || (int)adapter2.size() > FQ_MAX_ADAPTER)
        throw CliError("adapter longer than " + std::to_string(FQ_MAX_ADAPTER) + " bases", 2);
    if (cut_front && window_front < 1) throw CliError("--cut_front_window 0 is undefined in the reference", 2);
    if (cut_tail && window_tail < 1) throw CliError("--cut_tail_window 0 is undefined in the reference", 2);
    if (cut_right && window_right < 1) throw CliError("--cut_right_window 0 is undefined in the reference", 2);
    if (polyg && (polyg_min_len < 1 && paired())) throw CliError("polyG one-mismatch period must be >= 1", 2);
    if (polyg && !paired() && polyg_one_per < 1) throw CliError("polyG one-mismatch period must be >= 1", 2);
    if (polyx && polyx_one_per < 1) throw CliError("polyX one-mismatch period must be >= 1", 2);
}

std::vector<int> Options::device_list() const {
    if (devices.empty()) return {device};
    std::vector<int> out;
    size_t i = 0;
    while (i <= devices.size()) {
        const size_t j = std::min(devices.find(',', i), devices.size());
        long long v = 0;
        if (!cast_signed(devices.substr(i, j - i), v) || v < 0 || v > 1023)
            throw std::runtime_error("--devices must be a comma-separated list of device ids, got '" + devices + "'");
        out.push_back((int)v);
        i = j + 1;
    }
    return out;
}

fq_params Options::to_params(int max_cycles) const {
    fq_params p;
    std::memset(&p, 0, sizeof p);
    p.paired = paired() ? 1 : 0;
    p.trim_front1 = front1;
    p.trim_tail1 = tail1;
    p.trim_front2 = front2;
    p.trim_tail2 = tail2;
    p.cut_front = cut_front;
    p.cut_right = cut_right;
    p.cut_tail = cut_tail;
    p.cut_front_window = window_front;
    p.cut_right_window = window_right;
    p.cut_tail_window = window_tail;
    p.cut_front_quality = quality_front;
    p.cut_right_quality = quality_right;
    p.cut_tail_quality = quality_tail;
    p.polyg_enabled = polyg;
    if (paired()) {
        // PairEndProcessor passes (maxMismatch, allowedOneMismatchForEach, minLen) as
        // (compareReq, maxMismatch, allowedOneMismatchForEach): src/peprocessor.cpp:297 vs src/polyx.h:28
        p.polyg_compare_req = polyg_max_mismatch;
        p.polyg_max_mismatch = polyg_one_per;
        p.polyg_one_mismatch_per = polyg_min_len;
    } else {  // src/seprocessor.cpp:317
        p.polyg_compare_req = polyg_min_len;
        p.polyg_max_mismatch = polyg_max_mismatch;
        p.polyg_one_mismatch_per = polyg_one_per;
    }
    p.polyx_enabled = polyx;
    p.polyx_mask = 0;
    for (int b = 0; b < 5; ++b)
        if (polyx_chars.find("ATCGN"[b]) != std::string::npos) p.polyx_mask |= 1 << b;
    p.polyx_compare_req = polyx_min_len;
    p.polyx_max_mismatch = polyx_max_mismatch;
    p.polyx_one_mismatch_per = polyx_one_per;
    p.adapter_trimming = adapter_trimming;
    p.adapter1_len = (int)adapter1.size();
    p.adapter2_len = (int)adapter2.size();
    std::memcpy(p.adapter1, adapter1.data(), adapter1.size());
    std::memcpy(p.adapter2, adapter2.data(), adapter2.size());
    p.overlap_diff_limit = overlap_diff_limit;
    p.overlap_require = overlap_require;
    p.insert_size_max = insert_size_max;
    p.max_len1 = max_len1;
    p.max_len2 = max_len2;
    p.merge_enabled = merge;
    p.discard_unmerged = discard_unmerged;
    p.qual_filter_enabled = qual_filter;
    p.low_qual_limit = low_qual_limit;
    p.low_qual_base_limit = low_qual_base_limit;
    p.n_base_limit = n_base_limit;
    p.avg_qual_limit = avg_qual;
    p.length_filter_enabled = length_filter;
    p.min_len = min_len;
    p.max_len = max_len;
    p.complexity_enabled = complexity_filter;
    p.complexity_threshold = complexity_threshold;
    p.max_cycles = max_cycles;
    p.correction_enabled = correction && paired();
    p.umi_front1 = umi_front(0);  // UmiProcessor::process, src/umiprocessor.cpp:28-62
    p.umi_front2 = umi_front(1);
    return p;
}

}  // namespace fqhost
