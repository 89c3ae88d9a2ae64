// html.cpp -- the HTML report: HtmlReporter::report / printSummary / reportDuplication
// (reference src/htmlreporter.cpp:23-370), Stats::reportHtmlQuality / reportHtmlContents
// (src/stats.cpp:631-806) and FilterResult::reportHtmlBasic / reportAdaptersHtml* /
// reportPolyXTrimHtml (src/filterresult.cpp:223-376).
//
// The reference builds a DOM with the vendored CTML library and prints it on one line.  HNode is
// a small DOM with the same printing rules: `tag.class#id` selectors, class then id then the
// other attributes in the iteration order of a std::unordered_map (insertion sequence and hash
// are the same as the reference's, so the order is too), text children printed verbatim.
#include <chrono>
#include <cstdio>
#include <ctime>
#include <numeric>
#include <sstream>
#include <unordered_map>

#include "report.h"

namespace fqhost {
namespace {

struct HNode {
    bool text = false;
    std::string name, id, content;
    std::vector<std::string> classes;
    std::unordered_map<std::string, std::string> attrs;
    bool close = true;
    std::vector<HNode> kids;

    HNode() = default;
    explicit HNode(const std::string& sel) { set_name(sel); }
    HNode(const std::string& sel, const std::string& t) {
        set_name(sel);
        add_text(t);
    }
    static HNode make_text(const std::string& t) {
        HNode n;
        n.text = true;
        n.content = t;
        return n;
    }
    HNode& attr(const std::string& k, const std::string& v) {
        if (k == "id") {
            id = v;
        } else if (k == "class") {
            classes.clear();
            std::istringstream in(v);
            std::string c;
            while (std::getline(in, c, ' ')) classes.push_back(c);
        } else {
            attrs[k] = v;
        }
        return *this;
    }
    HNode& add(const HNode& c) {
        kids.push_back(c);
        return *this;
    }
    HNode& add_text(const std::string& t) { return add(make_text(t)); }

    // "name.class1.class2#id": the name ends at the first '.' or '#'
    void set_name(const std::string& sel) {
        const size_t cut = std::min(sel.find('.'), sel.find('#'));
        name = sel.substr(0, cut);
        if (cut == std::string::npos) return;
        int state = 0;  // 0 none, 1 class, 2 id
        std::string tmp;
        for (size_t i = cut; i < sel.size(); ++i) {
            const char c = sel[i];
            if (state == 0) {
                state = c == '.' ? 1 : c == '#' ? 2 : 0;
                continue;
            }
            if (c == '.' || c == '#') {
                if (state == 1) classes.push_back(tmp);
                else id = tmp;
                tmp.clear();
                state = c == '.' ? 1 : 2;
                continue;
            }
            tmp += c;
        }
        if (!tmp.empty()) {
            if (state == 1) classes.push_back(tmp);
            else if (state == 2) id = tmp;
        }
    }
    void print(std::string& out) const {
        if (text) {
            out += content;
            return;
        }
        out += "<" + name;
        if (!classes.empty()) {
            out += " class=\"";
            for (size_t i = 0; i < classes.size(); ++i) out += (i ? " " : "") + classes[i];
            out += "\"";
        }
        if (!id.empty()) out += " id=\"" + id + "\"";
        for (const auto& a : attrs) out += " " + a.first + "=\"" + a.second + "\"";
        out += ">";
        if (!close) return;
        for (const HNode& k : kids) k.print(out);
        out += "</" + name + ">";
    }
};

// std::to_string(double): "%f"
std::string fstr(double v) {
    char b[512];
    std::snprintf(b, sizeof b, "%f", v);
    return b;
}

// operator<< on a std::stringstream with default flags
template <class T>
std::string sstr(const T& v) {
    std::ostringstream s;
    s << v;
    return s.str();
}

template <class T>
HNode row2(const std::string& key, const T& val) {  // htmlutil::make2ColRowNode
    HNode r("tr");
    r.add(HNode("td.col1", key));
    r.add(HNode("td.col2", sstr(val)));
    return r;
}

// Stats::list2string (src/stats.h:216-225)
template <class T>
std::string list2string(const T* v, int n) {
    std::ostringstream s;
    for (int i = 0; i < n; ++i) {
        s << v[i];
        if (i < n - 1) s << ",";
    }
    return s.str();
}

std::string replace_all(std::string s, const std::string& a, const std::string& b) {
    std::string r;
    size_t las = 0, cur = 0;
    while ((cur = s.find(a, cur)) != std::string::npos) {
        r += s.substr(las, cur - las) + b;
        cur += a.size();
        las = cur;
    }
    return r + s.substr(las);
}

// the x positions of a curve (src/stats.cpp:640-667): every cycle, or for reads > 300 cycles the
// first 40 then every 5 % step (the y values are still the first `total` points, as there)
std::vector<int> curve_x(int cycles) {
    std::vector<int> x;
    if (cycles <= 300) {
        for (int i = 0; i < cycles; ++i) x.push_back(i + 1);
        return x;
    }
    for (int i = 0; i < 40 && i < cycles; ++i) x.push_back(i + 1);
    double pos = 40;
    for (;;) {
        pos *= 1.05;
        if (pos >= cycles) break;
        x.push_back((int)pos);
    }
    if (x.back() != cycles) x.push_back(cycles);
    return x;
}

std::string layout_x(int cycles) {
    std::string s = "var layout={title:'', xaxis:{title:'position', tickmode: 'auto', nticks: '" + std::to_string(cycles / 5) + "'";
    if (cycles > 300) s += ",type:'log'";
    return s;
}

// Stats::reportHtmlQuality, src/stats.cpp:631-714
HNode stats_quality(const Summary& st, const std::string& filtering, const std::string& read) {
    const std::string sub = filtering + ": " + read + ": quality";
    const std::string div = replace_all(replace_all(sub, " ", "_"), ":", "_");
    const char* names[5] = {"A", "T", "C", "G", "Mean"};
    const char* colors[5] = {"rgba(128,128,0,1.0)", "rgba(128,0,128,1.0)", "rgba(0,255,0,1.0)", "rgba(0,0,255,1.0)",
                             "rgba(20,20,20,1.0)"};
    const std::vector<int> x = curve_x(st.cycles);
    const int total = (int)x.size();
    std::string js = "var data=[";
    for (int b = 0; b < 5; ++b) {
        js += "{";
        js += "x:[" + list2string(x.data(), total) + "],";
        js += "y:[" + list2string(st.qual_curves[b].data(), total) + "],";
        js += std::string("name: '") + names[b] + "',";
        js += "mode:'lines',";
        js += std::string("line:{color:'") + colors[b] + "', width:1}\n";
        js += "},";
    }
    js += "];\n";
    js += layout_x(st.cycles) + "},";
    js += "yaxis:{title:'quality', tickmode: 'auto', nticks: '20'";
    js += "}};\n";
    js += "Plotly.newPlot('plot_" + div + "', data, layout);\n";
    HNode sec("div.section_div");
    HNode title("div.subsection_title");
    HNode link("a", sub);
    link.attr("title", "click to hide/show");
    link.attr("onclick", "showOrHide('" + div + "')");
    title.add(link);
    sec.add(title);
    HNode id("div#" + div);
    id.add(HNode("div.sub_section_tips", "Value of each position will be shown on mouse over"));
    id.add(HNode("div.figure#plot_" + div));
    sec.add(id);
    HNode script("script");
    script.attr("type", "text/javascript");
    script.add_text(js);
    sec.add(script);
    return sec;
}

// Stats::reportHtmlContents, src/stats.cpp:716-806
HNode stats_contents(const Summary& st, const std::string& filtering, const std::string& read) {
    const std::string sub = filtering + ": " + read + ": base contents";
    const std::string div = replace_all(replace_all(sub, " ", "_"), ":", "_");
    HNode sec("div.section_div");
    HNode title("div.subsection_title");
    HNode click("a", sub);
    click.attr("title", "click to hide/show");
    click.attr("onclick", "showOrHide('" + div + "')");
    title.add(click);
    sec.add(title);
    HNode id("div#" + div);
    id.add(HNode("div.sub_section_tips", "Value of each position will be shown on mouse over"));
    id.add(HNode("div.figure#plot_" + div));
    sec.add(id);
    HNode script("script");
    script.attr("type", "text/javascript");
    const char* names[6] = {"A", "T", "C", "G", "N", "GC"};
    const char* colors[6] = {"rgba(128,128,0,1.0)", "rgba(128,0,128,1.0)", "rgba(0,255,0,1.0)", "rgba(0,0,255,1.0)",
                             "rgba(255, 0, 0, 1.0)", "rgba(20,20,20,1.0)"};
    const std::vector<int> x = curve_x(st.cycles);
    const int total = (int)x.size();
    std::string js = "var data=[";
    for (int b = 0; b < 6; ++b) {
        const long count = b < 5 ? (long)st.base_contents[names[b][0] & 7]
                                 : (long)(st.base_contents['G' & 7] + st.base_contents['C' & 7]);
        std::string pct = fstr((double)count * 100.0 / (double)(long)st.bases);
        if (pct.size() > 5) pct = pct.substr(0, 5);
        js += "{";
        js += "x:[" + list2string(x.data(), total) + "],";
        js += "y:[" + list2string(st.content_curves[b].data(), total) + "],";
        js += std::string("name: '") + names[b] + "(" + pct + "%)',";
        js += "mode:'lines',";
        js += std::string("line:{color:'") + colors[b] + "', width:1}\n";
        js += "},";
    }
    js += "];\n";
    js += layout_x(st.cycles) + "}, yaxis:{title:'base content ratios'";
    js += ", tickmode: 'auto', nticks: '20', range: ['0.0', '1.0']";
    js += "}};\n";
    js += "Plotly.newPlot('plot_" + div + "', data, layout);\n";
    script.add_text(js);
    sec.add(script);
    return sec;
}

// FilterResult::reportAdaptersHtmlDetails, src/filterresult.cpp:267-306
HNode adapter_details(const AdapterCounts::Report& rep) {
    HNode table("table.summary_table");
    HNode head("tr");
    HNode c1("td.adapter_col", "Sequence");
    c1.attr("style", "font-size:14px;color:#ffffff;background:#556699");
    HNode c2("td.col2", "Occurences");
    c2.attr("style", "font-size:14px;color:#ffffff;background:#556699");
    head.add(c1).add(c2);
    table.add(head);
    const size_t total = rep.total;
    if (total == 0) return table;
    const double dt = (double)total;
    size_t reported = 0;
    for (auto& e : rep.top) {
        if (e.second / dt < 0.01) continue;
        HNode r("tr");
        r.add(HNode("td.adapter_col", e.first));
        r.add(HNode("td.col2", std::to_string(e.second) + "(" + fstr(e.second * 100.0 / dt) + "%)"));
        table.add(r);
        reported += e.second;
    }
    const size_t unreported = total - reported;
    if (unreported > 0)
        table.add(row2(reported == 0 ? "all adapter sequences" : "other adapter sequences",
                       std::to_string(unreported) + "(" + fstr(unreported * 100.0 / dt) + "%)"));
    return table;
}

// HtmlReporter::reportDuplication, src/htmlreporter.cpp:240-305
HNode duplication(const Options& o, const HostAcc& a) {
    const int total = std::max(0, o.dup_hist_size - 2);
    std::vector<long> x((size_t)total);
    std::vector<double> pct((size_t)total, 0.0), gc((size_t)total);
    auto hist = [&](int i) { return i < (int)a.dup_hist.size() ? a.dup_hist[(size_t)i] : 0; };
    auto mean_gc = [&](int i) {
        const uint64_t n = hist(i);
        return (int)n > 0 ? (double)a.dup_gc_sum[(size_t)i] / 255.0 / (int)n : 0.0;
    };
    double all = 0;
    for (int i = 0; i < total; ++i) {
        x[(size_t)i] = i + 1;
        all += (double)hist(i + 1);
    }
    if (all > 0)
        for (int i = 0; i < total; ++i) pct[(size_t)i] = (double)hist(i + 1) * 100.0 / all;
    int max_gc = total;
    for (int i = 0; i < total; ++i) {
        gc[(size_t)i] = mean_gc(i + 1) * 100.0;
        if (pct[(size_t)i] <= 0.05 && max_gc == total) max_gc = i;
    }
    const double rate = a.dup_total == 0 ? 0.0 : (double)a.dup_dups / (double)a.dup_total;
    std::string js = "var data=[";
    js += "{";
    js += "x:[" + list2string(x.data(), total) + "],";
    js += "y:[" + list2string(pct.data(), total) + "],";
    js += "name: 'Read percent (%)  ',";
    js += "type:'bar',";
    js += "line:{color:'rgba(128,0,128,1.0)', width:1}\n";
    js += "},";
    js += "{";
    js += "x:[" + list2string(x.data(), max_gc) + "],";
    js += "y:[" + list2string(gc.data(), max_gc) + "],";
    js += "name: 'Mean GC ratio (%)  ',";
    js += "mode:'lines',";
    js += "line:{color:'rgba(255,0,128,1.0)', width:2}\n";
    js += "}";
    js += "];\n";
    js += "var layout={title:'duplication rate (" + fstr(rate * 100.0) +
          "%)', xaxis:{title:'duplication level'}, yaxis:{title:'Read percent (%) & GC ratio'}};\n";
    js += "Plotly.newPlot('plot_duplication', data, layout);\n";
    HNode sec("div.section_div");
    HNode title("div.section_title");
    title.attr("onclick", "showOrHide('duplication')");
    HNode link("a", "Duplication");
    link.attr("name", "summary");
    title.add(link);
    sec.add(title);
    HNode id("div#duplication");
    HNode figid("div#duplication_figure");
    HNode fig("div.figure");
    fig.attr("id", "plot_duplication").attr("style", "height:400px;");
    figid.add(fig);
    id.add(figid);
    HNode script("script");
    script.attr("type", "text/javascript");
    script.add_text(js);
    sec.add(id);
    sec.add(script);
    return sec;
}

HNode section_title(const std::string& text, const std::string& div) {
    HNode t("div.section_title", text);
    t.attr("onclick", "showOrHide('" + div + "')");
    HNode link("a");
    link.attr("name", "summary");
    t.add(link);
    return t;
}

HNode subsection(const std::string& text, const std::string& div) {
    HNode s("div.subsection_title", text);
    s.attr("onclick", "showOrHide('" + div + "')");
    return s;
}

}  // namespace

std::string html_time_now() {  // htmlutil::getCurrentSystemTime, src/htmlutil.h:58-66
    const std::time_t tt = std::chrono::system_clock::to_time_t(std::chrono::system_clock::now());
    std::tm tmv;
    localtime_r(&tt, &tmv);
    char d[60] = {0};
    std::snprintf(d, sizeof d, "%d-%02d-%02d      %02d:%02d:%02d", tmv.tm_year + 1900, tmv.tm_mon + 1, tmv.tm_mday,
                  tmv.tm_hour, tmv.tm_min, tmv.tm_sec);
    return d;
}

std::string build_html(const Options& o, const HostAcc& a, const AdapterCounts& ac, const std::string& now) {
    const bool pe = o.paired();
    const Summary pre1 = summarize(a, 0), post1 = summarize(a, 2);
    Summary pre2, post2;
    if (pe) {
        pre2 = summarize(a, 1);
        post2 = summarize(a, 3);
    }
    HNode head("head"), body("body");
    // printHeader, src/htmlreporter.cpp:307-370
    HNode meta("meta");
    meta.attr("http-equiv", "content-type");
    meta.attr("content", "text/html;charset=utf-8");
    meta.close = false;
    head.add(meta);
    head.add(HNode("title", "Fastq Preprocess Report"));
    HNode js_src("script");
    js_src.attr("src", "https://cdn.plot.ly/plotly-latest.min.js");
    HNode js_fn("script");
    js_fn.attr("type", "text/javascript");
    for (const char* t : {"function showOrHide(divname) {\n", "  div = document.getElementById(divname);\n",
                          "  if(div.style.display == 'none')\n", "     div.style.display = 'block';\n", "  else\n",
                          "     div.style.display = 'none';\n", "}\n"})
        js_fn.add_text(t);
    head.add(js_src);
    head.add(js_fn);
    HNode css("style");
    css.attr("type", "text/css");
    for (const char* t :
         {"td {border:1px solid #dddddd;padding:5px;font-size:12px;}\n",
          "table {border:1px solid #999999;padding:2x;border-collapse:collapse; width:800px}\n",
          ".col1 {width:240px; font-weight:bold;}\n", ".adapter_col {width:500px; font-size:10px;}\n",
          "img {padding:30px;}\n", "#menu {font-family:Consolas, 'Liberation Mono', Menlo, Courier, monospace;}\n",
          "#menu a {color:#0366d6; font-size:18px;font-weight:600;line-height:28px;text-decoration:none;",
          "font-family:-apple-system, BlinkMacSystemFont, 'Segoe UI', Helv  etica, Arial, sans-serif, 'Apple Color "
          "Emoji', 'Segoe UI Emoji', 'Segoe UI Symbol'}\n",
          "a:visited {color: #999999}\n", ".alignleft {text-align:left;}\n", ".alignright {text-align:right;}\n",
          ".figure {width:800px;height:600px;}\n", ".header {color:#ffffff;padding:1px;height:20px;background:#000000;}\n",
          ".section_title {color:#ffffff;font-size:20px;padding:5px;text-align:left;background:#663355; "
          "margin-top:10px;}\n",
          ".subsection_title {font-size:16px;padding:5px;margin-top:10px;text-align:left;color:#663355}\n",
          "#container {text-align:center;padding:3px 3px 3px 10px;font-family:Arail,'Liberation Mono', Menlo, "
          "Courier, monospace;}\n",
          ".menu_item {text-align:left;padding-top:5px;font-size:18px;}\n",
          ".highlight {text-align:left;padding-top:30px;padding-bottom:30px;font-size:20px;line-height:35px;}\n",
          "#helper {text-align:left;border:1px dotted #fafafa;color:#777777;font-size:12px;}\n",
          "#footer {text-align:left;padding:15px;color:#ffffff;font-size:10px;background:#663355;font-family:Arail,'"
          "Liberation Mono', Menlo, Courier, monospace;}\n",
          ".kmer_table {text-align:center;font-size:8px;padding:2px;}\n",
          ".kmer_table td{text-align:center;font-size:8px;padding:0px;color:#ffffff}\n",
          ".sub_section_tips {color:#999999;font-size:10px;padding-left:5px;padding-bottom:3px;}\n"})
        css.add_text(t);
    head.add(css);

    // printSummary, src/htmlreporter.cpp:97-238
    long pre_reads = (long)(pre1.reads + pre2.reads), pre_bases = (long)(pre1.bases + pre2.bases);
    long pre_q20 = (long)(pre1.q20 + pre2.q20), pre_q30 = (long)(pre1.q30 + pre2.q30), pre_gc = (long)(pre1.gc + pre2.gc);
    long post_reads = (long)(post1.reads + post2.reads), post_bases = (long)(post1.bases + post2.bases);
    long post_q20 = (long)(post1.q20 + post2.q20), post_q30 = (long)(post1.q30 + post2.q30);
    long post_gc = (long)(post1.gc + post2.gc);
    auto rate = [](long n, long d) { return d == 0 ? 0.0 : (double)n / d; };
    const double pre_q20r = rate(pre_q20, pre_bases), pre_q30r = rate(pre_q30, pre_bases), pre_gcr = rate(pre_gc, pre_bases);
    const double post_q20r = rate(post_q20, post_bases), post_q30r = rate(post_q30, post_bases);
    const double post_gcr = rate(post_gc, post_bases);
    std::string seqinfo = pe ? "paired end" : "single end";
    if (pe) seqinfo += " (" + std::to_string(pre1.cycles) + " cycles + " + std::to_string(pre2.cycles) + " cycles)";
    else seqinfo += " (" + std::to_string(pre1.cycles) + " cycles)";
    HNode h1("h1");
    h1.attr("style", "text-align:left");
    HNode h1a("a");
    h1a.attr("style", "color:#663355;text-decoration:none;").add_text("Fastq Report");
    h1.add(h1a);
    head.add(h1);
    HNode summary_sec("div.section_div");
    HNode summary_title("div.section_title");
    summary_title.attr("onclick", "showOrHide('summary')");
    HNode summary_link("a", "Summary");
    summary_link.attr("name", "summary");
    summary_title.add(summary_link);
    summary_sec.add(summary_title);
    HNode summary("div#summary");
    HNode general_id("div#general");
    HNode general("table.summary_table");
    general.add(row2("Sequencing", seqinfo));
    if (pe) {
        int peak = 0;
        long maxc = -1;
        for (int i = 0; i < a.insert_size_max(); ++i)
            if ((long)a.head()[FQ_ACC_INSERT + i] > maxc) {
                peak = i;
                maxc = (long)a.head()[FQ_ACC_INSERT + i];
            }
        general.add(row2("Insert Size Peak", peak));
    }
    if (o.adapter_trimming) {
        if (!o.detected_adapter1.empty()) general.add(row2("Detected Read1 Adapter", o.detected_adapter1));
        if (!o.detected_adapter2.empty()) general.add(row2("Detected Read2 Adapter", o.detected_adapter2));
    }
    general_id.add(general);
    summary.add(subsection("General", "general"));
    summary.add(general_id);
    HNode pre_id("div#before_filtering_summary");
    HNode pre_t("table.summary_table");
    pre_t.add(row2("Total Reads", pre_reads));
    pre_t.add(row2("Total Bases", pre_bases));
    pre_t.add(row2("Q20 Bases", std::to_string(pre_q20) + "(" + fstr(pre_q20r * 100) + "%)"));
    pre_t.add(row2("Q30 Bases", std::to_string(pre_q30) + "(" + fstr(pre_q30r * 100) + "%)"));
    pre_t.add(row2("GC Content", fstr(pre_gcr * 100) + "%"));
    pre_t.add(row2("Read1 Mean Length", pre1.mean_length()));
    if (pe) pre_t.add(row2("Read2 Mean Length", pe ? pre2.mean_length() : 0));
    if (o.adapter_trimming) {
        size_t with = ac.report(0).total;
        double r = pe ? with * 1.0 / pre_reads * 2 : with * 1.0 / pre_reads;
        pre_t.add(row2("Read1 Adapters Left", std::to_string(with) + "(" + fstr(r * 100) + "%)"));
        if (pe) {
            with = ac.report(1).total;
            r = with * 1.0 / pre_reads * 2;
            pre_t.add(row2("Read2 Adapters Left", std::to_string(with) + "(" + fstr(r * 100) + "%)"));
        }
    }
    pre_id.add(pre_t);
    summary.add(subsection("Before Filtering", "before_filtering_summary"));
    summary.add(pre_id);
    HNode post_id("div#after_filtering_summary");
    HNode post_t("table.summary_table");
    post_t.add(row2("Total Reads", post_reads));
    post_t.add(row2("Total Bases", post_bases));
    post_t.add(row2("Q20 Bases", std::to_string(post_q20) + "(" + fstr(post_q20r * 100) + "%)"));
    post_t.add(row2("Q30 Bases", std::to_string(post_q30) + "(" + fstr(post_q30r * 100) + "%)"));
    post_t.add(row2("GC Content", fstr(100 * post_gcr) + "%"));
    post_t.add(row2("Read1 Mean Length", post1.mean_length()));
    if (pe) post_t.add(row2("Read2 Mean Length", post2.mean_length()));
    post_id.add(post_t);
    summary.add(subsection("After filtering", "after_filtering_summary"));
    summary.add(post_id);
    // FilterResult::reportHtmlBasic(totalReads, totalBases), called with (preTotalBases,
    // preTotalReads) (src/htmlreporter.cpp:221): the names are swapped on the way in
    const size_t arg_reads = (size_t)pre_bases, arg_bases = (size_t)pre_reads;
    HNode ft("table.summary_table");
    auto pctrow = [&](const std::string& k, uint64_t v, size_t den) {
        ft.add(row2(k, std::to_string(v) + "(" + fstr(v * 100.0 / den) + "%)"));
    };
    pctrow("Reads Passed Filters", a.filter(FQ_PASS_FILTER), arg_bases);
    pctrow("Low Quality Reads", a.filter(FQ_FAIL_QUALITY), arg_bases);
    pctrow("Too Many N Reads", a.filter(FQ_FAIL_N_BASE), arg_bases);
    if (o.correction) {
        pctrow("Corrected Reads", a.tail(FQ_ACC_TAIL_CORRECTED_READS), arg_reads);
        pctrow("Corrected Bases", a.tail(FQ_ACC_TAIL_CORRECTED_BASES), arg_bases);
    }
    if (o.complexity_filter) pctrow("Low Complexity Reads", a.filter(FQ_FAIL_COMPLEXITY), arg_reads);
    if (o.length_filter) {
        pctrow("Too Short Reads", a.filter(FQ_FAIL_LENGTH), arg_reads);
        if (o.max_len > 0) pctrow("Too Long Reads", a.filter(FQ_FAIL_TOO_LONG), arg_reads);
    }
    HNode fr_id("div#filtering_result");
    fr_id.add(ft);
    summary.add(subsection("Filtering Results", "filtering_result"));
    summary.add(fr_id);
    body.add(summary_sec);
    body.add(summary);
    if (o.adapter_trimming) {  // FilterResult::reportAdaptersHtmlSummary, src/filterresult.cpp:329-357
        HNode sec("div.section_div");
        sec.add(section_title("Adapters", "adapters"));
        HNode ids("div#adapters");
        HNode a1("div#read1_adapters");
        a1.add(adapter_details(ac.report(0)));
        ids.add(subsection("Adapter or bad ligation of read1", "read1_adapters"));
        ids.add(a1);
        if (pe) {
            HNode a2("div#read2_adapters");
            a2.add(adapter_details(ac.report(1)));
            ids.add(subsection("Adapter or bad ligation of read2", "read2_adapters"));
            ids.add(a2);
        }
        sec.add(ids);
        body.add(sec);
    }
    if (o.polyg || o.polyx) {  // FilterResult::reportPolyXTrimHtml, src/filterresult.cpp:359-376
        HNode sec("div.section_div");
        sec.add(section_title("PolyX Trimming", "polyx"));
        HNode id("div#polyx");
        HNode t("table.summary_table");
        int rsum = 0, bsum = 0;  // std::accumulate(..., 0): int
        for (int b = 0; b < 5; ++b) {
            rsum += (int)a.head()[FQ_ACC_POLYX_READS + b];
            bsum += (int)a.head()[FQ_ACC_POLYX_BASES + b];
        }
        t.add(row2("TotalPolyXTrimmedReads", rsum));
        t.add(row2("TotalPolyXTrimmedBases", bsum));
        const char* nc = "ATCGN";
        for (int b = 0; b < 5; ++b)
            t.add(row2(std::string("ReadsTrimmedByPoly") + nc[b], a.head()[FQ_ACC_POLYX_READS + b]));
        for (int b = 0; b < 5; ++b)
            t.add(row2(std::string("BasesTrimmedByPoly") + nc[b], a.head()[FQ_ACC_POLYX_BASES + b]));
        id.add(t);
        sec.add(id);
        body.add(sec);
    }
    if (o.dup) body.add(duplication(o, a));

    // HtmlReporter::report, src/htmlreporter.cpp:23-95
    HNode pre_sec("div.section_div");
    HNode pre_title("div.section_title");
    pre_title.attr("onclick", "showOrHide('before_filtering')");
    HNode pre_link("a", "Before filtering");
    pre_link.attr("name", "summary");
    pre_title.add(pre_link);
    pre_sec.add(pre_title);
    HNode pre_div("div#before_filtering");
    pre_div.add(stats_quality(pre1, "Before filtering", "read1")).add(stats_contents(pre1, "Before filtering", "read1"));
    if (pe)
        pre_div.add(stats_quality(pre2, "Before filtering", "read2")).add(stats_contents(pre2, "Before filtering", "read2"));
    body.add(pre_sec);
    body.add(pre_div);
    HNode post_sec("div.section_div");
    HNode post_title("div.section_title");
    post_title.attr("onclick", "showOrHide('after_filtering')");
    HNode post_link("a", "After filtering");
    post_link.attr("name", "summary");
    post_title.add(post_link);
    post_sec.add(post_title);
    HNode post_div("div#after_filtering");
    post_div.add(stats_quality(post1, "After filtering", "read1")).add(stats_contents(post1, "After filtering", "read1"));
    if (pe)
        post_div.add(stats_quality(post2, "After filtering", "read2")).add(stats_contents(post2, "After filtering", "read2"));
    post_sec.add(post_div);
    body.add(post_sec);
    HNode sw("div#section_div");
    HNode sw_title("div.section_title");
    sw.attr("onclick", "showOrHide('software')");
    HNode sw_link("a", "Software Environment");
    sw_link.attr("name", "summary");
    sw_title.add(sw_link);
    sw.add(sw_title);
    HNode sw_id("div#software");
    HNode sw_t("table.summary_table");
    sw_t.add(row2("Version", o.version));
    sw_t.add(row2("Command", o.command));
    sw_t.add(row2("CWD", o.cwd));
    sw_id.add(sw_t);
    body.add(sw);
    body.add(sw_id);
    body.add(HNode("div#footer", "Fqtool Report @ " + now));

    HNode html("html");
    html.add(head);
    html.add(body);
    std::string out = "<!DOCTYPE html>";
    html.print(out);
    return out;
}

}  // namespace fqhost
