// processor.h -- the host pipeline around the engine: the reference's
// Processor / PairEndProcessor / SingleEndProcessor plumbing (src/processor.cpp:10-19,
// src/peprocessor.cpp:99-247, src/seprocessor.cpp) with the per-pack loop body delegated to the
// gfx950 engine through the C-ABI (include/fqengine.h).
//
// Threads: one reader (FASTQ parse + pack build), the engine caller (H2D, kernels, D2H, output
// formatting in input order -- identical to the reference run with -w 1), one writer per output
// file.  Packs are processed strictly in input order.
#pragma once

#include <memory>
#include <functional>
#include <string>

#include "fastq.h"
#include "options.h"
#include "report.h"

namespace fqhost {

// Output text of one pack, per destination (src/peprocessor.cpp:262-269), as consecutive blocks
// (one per formatting range; a gzip output writes each block as one member)
struct PackOutput {
    std::vector<std::string> out1, out2, unpaired1, unpaired2, failed, merged;
};

class AsyncWriter;

// The output files of a run and the rule for which text goes where
// (PairEndProcessor::initOutput / SingleEndProcessor::initOutput and the tail of the pack loops,
// src/peprocessor.cpp:39-61, :457-492; src/seprocessor.cpp).  Each file has its own writer thread.
class OutputSet {
   public:
    explicit OutputSet(const Options& o, Pool* pool = nullptr);  // pool: gzip compression
    ~OutputSet();
    void write(PackOutput&& out);
    // out1 / out2 text as is (waits until both writers have taken it)
    // queue engine-assembled output text of both mates; `done` runs once both are written
    void write_text(const char* t1, size_t n1, const char* t2, size_t n2, std::function<void()> done);
    // the same as byte ranges (plain outputs: writev); the ranges stay valid until `done` runs
    void write_text_segs(const std::vector<iovec>& s1, const std::vector<iovec>& s2, std::function<void()> done);
    bool plain_pair_outputs() const;  // out1 / out2 (those that exist) are not gzip
    // -m: a text pack's merged stream (the merged output; out1 / out2 get nothing)
    void write_merged_text(const char* t, size_t n, std::function<void()> done);
    void close();  // flushes and closes every file

   private:
    bool paired_;
    std::unique_ptr<AsyncWriter> w1_, w2_, wu1_, wu2_, wf_, wm_;
};

// Builds the output text of one processed pack from the engine's per-read records, exactly as
// the loop body of processPairEnd / processSingleEnd appends to its strings.
// With a pool, ranges of the pack are formatted in parallel into consecutive blocks; `cuts`
// (optional, ascending, 0 .. n) fixes the block boundaries.
void format_pack(const Options& o, const Pack& pk, const fq_read_result* res, PackOutput& out, Pool* pool = nullptr,
                 const std::vector<int>* cuts = nullptr);

class SplitSink;

// Where a run's output goes: the regular files (OutputSet), or with -s / -S the numbered split
// files of ThreadConfig (src/threadconfig.cpp:88-137).  Packs must arrive in input order.
class Sink {
   public:
    Sink(const Options& o, Pool* pool);
    ~Sink();
    void consume(const Pack& pk, const fq_read_result* res);  // format + write one processed pack
    // write a text pack's engine-assembled output (no split); `done` runs (on a writer thread) once
    // the pack's text is written
    void consume_text(const Pack& pk, std::function<void()> done);
    bool plain_pair_outputs() const;  // text packs may go out as byte ranges (Pack::zc)
    void close();

   private:
    const Options& o_;
    Pool* pool_;
    std::unique_ptr<OutputSet> outs_;
    std::unique_ptr<SplitSink> split_;
    uint64_t pairs_ = 0;  // pairs (reads) consumed so far: the next pack's first global index
    bool merge_ = false;  // -m (PE): text packs carry the merged stream
};

// Before the engine call: per-pair index-filter flags (Filter::filterByIndex) when enabled.
void prepare_pack(const Options& o, Pack& pk, Pool* pool = nullptr);
// After it (-c): pairs with FQ_RF_CORRECTED records read corrected copies of their text.
void apply_corrections(const Options& o, Pack& pk, const fq_read_result* res, Pool* pool = nullptr);

// OverlapAnalysis::merge name rule (src/overlapanalysis.cpp:93-101)
std::string merged_name(const std::string& name, int len1, int len2);

// CLI parse + Options::update/validate + the Evaluator pre-pass (read length estimate,
// PE adapter detection), src/main.cpp:100-143.  Throws CliError / std::runtime_error.
Options prepare_options(int argc, char** argv, bool detect_adapters = true);

// The whole tool: returns the process exit code.
// exit_when_done: the command-line binary ends the process right after the outputs and reports
// are written and the summary logged (_exit, no teardown of page-locked buffers, engines, pool);
// in-process callers (fqh_run) get the return code as usual.
int run_tool(int argc, char** argv, bool exit_when_done = false);

}  // namespace fqhost
