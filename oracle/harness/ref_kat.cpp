// Known-answer-test harness: drives the UNMODIFIED reference per-read functions
// (compiled from /root/reference/src by oracle/Makefile.ref) on crafted inputs and
// prints their results, so the CPU restatement (oracle/fq_oracle.c) and the HIP
// kernels can be pinned against the reference itself.  Built and run only in the
// development container; its outputs are committed as tests/golden/kat_*.tsv.
//
// Input (stdin): one case per line, TAB separated:
//   kind  params  seq1  qual1  seq2  qual2  extra
// Output (stdout): the same case id followed by the reference's answer.
// '~' encodes an empty string in both directions.
#include <cstdio>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>
#include "options.h"
#include "read.h"
#include "filter.h"
#include "polyx.h"
#include "overlapanalysis.h"
#include "adaptertrimmer.h"
#include "filterresult.h"

static std::vector<std::string> splitTab(const std::string& s) {
    std::vector<std::string> out;
    std::string cur;
    for (char c : s) {
        if (c == '\t') { out.push_back(cur); cur.clear(); }
        else cur.push_back(c);
    }
    out.push_back(cur);
    for (auto& f : out) if (f == "~") f.clear();
    return out;
}

static std::vector<double> nums(const std::string& s) {
    std::vector<double> v;
    std::stringstream ss(s);
    std::string tok;
    while (std::getline(ss, tok, ',')) v.push_back(std::stod(tok));
    return v;
}

static std::string enc(const std::string& s) { return s.empty() ? std::string("~") : s; }

int main() {
    std::string line;
    long id = 0;
    while (std::getline(std::cin, line)) {
        if (line.empty() || line[0] == '#') continue;
        std::vector<std::string> f = splitTab(line);
        while (f.size() < 7) f.push_back("");
        const std::string& kind = f[0];
        Options opt;
        std::ostringstream out;
        out << id++ << '\t' << kind << '\t';
        if (kind == "pass") {
            // qualEnabled,lenEnabled,lowQualLimitRaw,lowQualBaseLimit,nBaseLimit,avgQual,minLen,maxLen,complexEnabled,complexThr
            std::vector<double> p = nums(f[1]);
            opt.qualFilter.enabled = p[0] != 0;
            opt.lengthFilter.enabled = p[1] != 0;
            opt.qualFilter.lowQualityLimit = (int)p[2] + 33;
            opt.qualFilter.lowQualityBaseLimit = (int)p[3];
            opt.qualFilter.nBaseLimit = (int)p[4];
            opt.qualFilter.averageQualityLimit = p[5];
            opt.lengthFilter.minReadLength = (int)p[6];
            opt.lengthFilter.maxReadLength = (int)p[7];
            opt.complexityFilter.enabled = p[8] != 0;
            opt.complexityFilter.threshold = p[9];
            Filter flt(&opt);
            Read* r = f[2] == "NULL" ? NULL : new Read("@r", f[2], "+", f[3]);
            out << flt.passFilter(r);
            delete r;
        } else if (kind == "cut") {
            // front,tail,enFront,enRight,enTail,wF,wR,wT,qF,qR,qT
            std::vector<double> p = nums(f[1]);
            opt.qualitycut.enableFront = p[2] != 0;
            opt.qualitycut.enableRright = p[3] != 0;
            opt.qualitycut.enableTail = p[4] != 0;
            opt.qualitycut.windowSizeFront = (int)p[5];
            opt.qualitycut.windowSizeRight = (int)p[6];
            opt.qualitycut.windowSizeTail = (int)p[7];
            opt.qualitycut.qualityFront = (int)p[8];
            opt.qualitycut.qualityRight = (int)p[9];
            opt.qualitycut.qualityTail = (int)p[10];
            Filter flt(&opt);
            Read* r = new Read("@r", f[2], "+", f[3]);
            Read* res = flt.trimAndCut(r, (int)p[0], (int)p[1]);
            if (!res) out << "NULL";
            else out << enc(res->seq.seqStr) << '\t' << enc(res->quality);
            delete r;
        } else if (kind == "polyg") {
            // compareReq,maxMismatch,perN
            std::vector<double> p = nums(f[1]);
            FilterResult fr(&opt, false);
            Read* r = new Read("@r", f[2], "+", f[3]);
            PolyX::trimPolyG(r, (int)p[0], (int)p[1], (int)p[2], &fr);
            out << enc(r->seq.seqStr) << '\t' << fr.mTrimmedPolyXReads[3] << '\t'
                << fr.mTrimmedPolyXBases[3];
            delete r;
        } else if (kind == "polyx") {
            // params: compareReq,maxMismatch,perN ; extra = trimChr
            std::vector<double> p = nums(f[1]);
            FilterResult fr(&opt, false);
            Read* r = new Read("@r", f[2], "+", f[3]);
            PolyX::trimPolyX(r, f[6], (int)p[0], (int)p[1], (int)p[2], &fr);
            out << enc(r->seq.seqStr);
            for (int b = 0; b < 5; ++b)
                out << '\t' << fr.mTrimmedPolyXReads[b] << ',' << fr.mTrimmedPolyXBases[b];
            delete r;
        } else if (kind == "overlap") {
            // diffLimit,require
            std::vector<double> p = nums(f[1]);
            Read r1("@a", f[2], "+", f[3]);
            Read r2("@b", f[4], "+", f[5]);
            OverlapResult ov = OverlapAnalysis::analyze(&r1, &r2, (int)p[0], (int)p[1]);
            out << (ov.overlapped ? 1 : 0) << '\t' << ov.offset << '\t' << ov.overlapLen << '\t' << ov.diff;
        } else if (kind == "merge") {
            // params: diffLimit,require ; extra = read-1 name
            std::vector<double> p = nums(f[1]);
            Read r1(f[6], f[2], "+", f[3]);
            Read r2("@b", f[4], "+", f[5]);
            OverlapResult ov = OverlapAnalysis::analyze(&r1, &r2, (int)p[0], (int)p[1]);
            Read* m = ov.overlapped ? OverlapAnalysis::merge(&r1, &r2, ov) : NULL;
            if (!m) out << "NULL";
            else out << enc(m->name) << '\t' << enc(m->seq.seqStr) << '\t' << enc(m->quality);
            delete m;
        } else if (kind == "adseq") {
            // params: isR2 ; extra = adapter
            std::vector<double> p = nums(f[1]);
            FilterResult fr(&opt, true);
            Read* r = new Read("@r", f[2], "+", f[3]);
            std::string ad = f[6];
            bool isR2 = p[0] != 0;
            bool trimmed = AdapterTrimmer::trimBySequence(r, &fr, ad, isR2);
            std::map<std::string, size_t>& m = isR2 ? fr.mAdapter2Count : fr.mAdapter1Count;
            out << (trimmed ? 1 : 0) << '\t' << enc(r->seq.seqStr) << '\t' << fr.mTrimmedAdapterReads
                << '\t' << fr.mTrimmedAdapterBases << '\t';
            std::string rec;
            for (auto& e : m) rec += e.first;
            out << enc(rec);
            delete r;
        } else if (kind == "adov") {
            // params: diffLimit,require
            std::vector<double> p = nums(f[1]);
            FilterResult fr(&opt, true);
            Read r1("@a", f[2], "+", f[3]);
            Read r2("@b", f[4], "+", f[5]);
            OverlapResult ov = OverlapAnalysis::analyze(&r1, &r2, (int)p[0], (int)p[1]);
            bool trimmed = AdapterTrimmer::trimByOverlapAnalysis(&r1, &r2, &fr, ov);
            std::string a1, a2;
            for (auto& e : fr.mAdapter1Count) a1 += e.first;
            for (auto& e : fr.mAdapter2Count) a2 += e.first;
            out << (trimmed ? 1 : 0) << '\t' << enc(r1.seq.seqStr) << '\t' << enc(r2.seq.seqStr) << '\t'
                << fr.mTrimmedAdapterReads << '\t' << fr.mTrimmedAdapterBases << '\t' << enc(a1)
                << '\t' << enc(a2);
        } else {
            out << "UNKNOWN";
        }
        std::cout << out.str() << '\n';
    }
    return 0;
}
