// text_format.cpp -- native writers/readers of the reference's text formats.
//
//  * impact TSV lines (reference src/deep_impact/indexing/indexer.py:62-68):
//      ', '.join(f'{term}: {round(impact, 3)}') + '\n'  -- the number is the
//      repr of the double value of the rounded float32 (pytext.h repr_double).
//  * quantize_file (src/deep_impact/indexing/quantize.py:17-47): parse
//      'term: score' pairs, quantize on the GPU (di_quantize_f64 semantics),
//      keep values > 0, write 'term: val' lines.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <string_view>
#include <algorithm>
#include <thread>
#include <vector>

#include "di_common.h"
#include "pytext.h"

namespace di {
void launch_quantize_f64(const double *v, int64_t n, double max_given, int bits, int32_t *out,
                         unsigned long long *max_bits, hipStream_t s);
}

using namespace di;

extern "C" int di_format_impact_lines(const char *terms, const int64_t *term_off,
                                      const float *impacts, const int64_t *cu_doc_terms,
                                      int32_t n_docs, char *out, int64_t out_cap,
                                      int64_t *out_len) {
    return guard([&] {
        DI_REQUIRE(term_off && cu_doc_terms && out_len && n_docs >= 0, DI_EINVAL,
                   "null argument");
        std::string buf;
        const int64_t nt = cu_doc_terms[n_docs];
        buf.reserve((size_t)(term_off[nt] - term_off[0]) + (size_t)nt * 24 + (size_t)n_docs);
        for (int32_t d = 0; d < n_docs; ++d) {
            for (int64_t i = cu_doc_terms[d]; i < cu_doc_terms[d + 1]; ++i) {
                if (i > cu_doc_terms[d]) buf += ", ";
                buf.append(terms + term_off[i], (size_t)(term_off[i + 1] - term_off[i]));
                buf += ": ";
                py::repr_double((double)impacts[i], buf);
            }
            buf += '\n';
        }
        *out_len = (int64_t)buf.size();
        DI_REQUIRE(out && (int64_t)buf.size() <= out_cap, DI_ERANGE,
                   "output buffer too small: %lld bytes needed", (long long)buf.size());
        std::memcpy(out, buf.data(), buf.size());
    });
}

// run-file lines (reference src/utils/datasets.py RunFile.writelines, :305-324):
// f"{qid}\t{pid}\t{rank}\t{score}\n" for rank = 1.. over each query's (pid, score)
// list, queries in order, appended to the file.  Integer pids and scores (the quantized
// index).  Formatted on host_threads() threads (<= 16) in rounds of query groups.
namespace {
inline int dec_digits(uint32_t v) {
    int d = 1;
    while (v >= 10) v /= 10, ++d;
    return d;
}
inline char *put_dec(char *p, uint32_t v, int d) {
    for (int i = d - 1; i >= 0; --i) p[i] = (char)('0' + v % 10), v /= 10;
    return p + d;
}
}  // namespace

extern "C" int di_append_run_lines(const char *path, const char *qids, const int64_t *qid_off,
                                   int32_t n_q, const uint32_t *docs, const uint32_t *scores,
                                   const int32_t *counts, int32_t k) {
    return guard([&] {
        DI_REQUIRE(path && qid_off && n_q >= 0 && k > 0, DI_EINVAL, "bad argument");
        DI_REQUIRE(n_q == 0 || (qids && docs && scores && counts), DI_EINVAL, "null argument");
        for (int32_t q = 0; q < n_q; ++q)
            DI_REQUIRE(counts[q] >= 0 && counts[q] <= k, DI_ERANGE,
                       "query %d: count %d outside [0, %d]", q, counts[q], k);
        std::FILE *f = std::fopen(path, "ab");
        DI_REQUIRE(f, DI_EIO, "cannot open %s", path);
        // rounds of nt consecutive query groups: every thread formats its group into its
        // own (reused) buffer, then the buffers are written in order -- no buffer of
        // the whole batch (first-touching one costs more than formatting it)
        const int nt = std::max(1, std::min(host_threads(), 16));
        constexpr int32_t GROUP = 32;  // queries per thread and round
        std::vector<std::string> bufs((size_t)nt);
        bool ok = true;
        for (int32_t r0 = 0; r0 < n_q && ok; r0 += nt * GROUP) {
            auto work = [&](int t) {
                std::string &b = bufs[(size_t)t];
                b.clear();
                const int32_t q0 = std::min(n_q, r0 + t * GROUP), q1 = std::min(n_q, q0 + GROUP);
                char *p = nullptr;
                for (int pass = 0; pass < 2; ++pass) {  // bytes, then the lines
                    int64_t need = 0;
                    for (int32_t q = q0; q < q1; ++q) {
                        const char *id = qids + qid_off[q];
                        const size_t idn = (size_t)(qid_off[q + 1] - qid_off[q]);
                        const uint32_t *dq = docs + (int64_t)q * k, *sq = scores + (int64_t)q * k;
                        for (int32_t i = 0; i < counts[q]; ++i) {
                            const int d1 = dec_digits(dq[i]), d2 = dec_digits((uint32_t)i + 1),
                                      d3 = dec_digits(sq[i]);
                            if (pass == 0) {
                                need += (int64_t)idn + 4 + d1 + d2 + d3;
                                continue;
                            }
                            std::memcpy(p, id, idn);
                            p += idn;
                            *p++ = '\t';
                            p = put_dec(p, dq[i], d1);
                            *p++ = '\t';
                            p = put_dec(p, (uint32_t)i + 1, d2);
                            *p++ = '\t';
                            p = put_dec(p, sq[i], d3);
                            *p++ = '\n';
                        }
                    }
                    if (pass == 0) {
                        b.resize((size_t)need);
                        p = b.data();
                    }
                }
            };
            std::vector<std::thread> th;
            for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
            work(0);
            for (auto &x : th) x.join();
            for (auto &b : bufs)
                ok = ok && std::fwrite(b.data(), 1, b.size(), f) == b.size();
        }
        ok = (std::fclose(f) == 0) && ok;
        DI_REQUIRE(ok, DI_EIO, "short write to %s", path);
    });
}

namespace {

std::string read_all(const char *path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    DI_REQUIRE(f, DI_EIO, "cannot open %s", path);
    std::string s((size_t)f.tellg(), '\0');
    f.seekg(0);
    f.read(s.data(), (std::streamsize)s.size());
    return s;
}

}  // namespace

// quantize_file: two passes of the reference become parse-once + one GPU kernel.  The
// parse and the output formatting run on host_threads() threads over ranges of whole
// lines (the output is the ranges' text in order).
extern "C" int di_quantize_file(const char *input_path, const char *output_path, double max_val,
                                int32_t bits, int device, double *max_used) {
    return guard([&] {
        DI_REQUIRE(input_path, DI_EINVAL, "null argument");
        const std::string buf = read_all(input_path);
        const std::vector<size_t> cut = py::line_chunks(buf, 8 * host_threads());
        const int C = (int)cut.size() - 1;
        struct Part {
            std::vector<std::string_view> terms;
            std::vector<double> vals;
            std::vector<uint32_t> cu{0};
            std::string out;
        };
        std::vector<Part> P((size_t)std::max(C, 1));
        // for doc_id, line in enumerate(f): for t in line.strip().split(', '):
        //     term, score = t.strip().split(': ')         (quantize.py:21-22, :41-42)
        parallel_chunks(C, [&](int64_t c, int) {
            Part &pc = P[(size_t)c];
            std::vector<std::string_view> pieces, tv;
            int64_t ln = 0;  // lines of this range seen so far
            with_line_context([&] {
            py::for_each_line(std::string_view(buf).substr(cut[c], cut[c + 1] - cut[c]),
                              [&](std::string_view line) {
                ++ln;
                py::split(py::strip(line), ", ", pieces);
                for (auto t : pieces) {
                    py::split(py::strip(t), ": ", tv);
                    DI_REQUIRE(tv.size() == 2, DI_EFORMAT,
                               "'%.*s' is not 'term: score' (the reference raises ValueError)",
                               (int)std::min<size_t>(t.size(), 200), t.data());
                    double v;
                    DI_REQUIRE(py::parse_float(tv[1], &v), DI_EFORMAT,
                               "could not convert '%.*s' to float",
                               (int)std::min<size_t>(tv[1].size(), 64), tv[1].data());
                    pc.terms.push_back(tv[0]);
                    pc.vals.push_back(v);
                }
                pc.cu.push_back((uint32_t)pc.terms.size());
            });
            }, [&] { return py::count_lines(std::string_view(buf).substr(0, cut[c])) + ln; });
        });
        std::vector<int64_t> off((size_t)C + 1, 0);
        for (int c = 0; c < C; ++c) off[(size_t)c + 1] = off[(size_t)c] + (int64_t)P[(size_t)c].vals.size();
        const int64_t n = off[(size_t)C];
        std::vector<double> vals((size_t)std::max<int64_t>(n, 1));
        parallel_for(C, [&](int64_t lo, int64_t hi, int) {
            for (int64_t c = lo; c < hi; ++c) {
                auto &v = P[(size_t)c].vals;
                std::copy(v.begin(), v.end(), vals.begin() + off[(size_t)c]);
                std::vector<double>().swap(v);
            }
        });
        int prev = 0;
        DI_HIP(hipGetDevice(&prev));
        DI_HIP(hipSetDevice(device));
        DevBuf dv, dq, dm;
        dv.reserve((size_t)std::max<int64_t>(n, 1) * 8);
        dq.reserve((size_t)std::max<int64_t>(n, 1) * 4);
        dm.reserve(16);
        if (n) DI_HIP(hipMemcpy(dv.p, vals.data(), (size_t)n * 8, hipMemcpyHostToDevice));
        launch_quantize_f64(dv.as<double>(), n, max_val, bits, dq.as<int32_t>(),
                            dm.as<unsigned long long>(), nullptr);
        std::vector<int32_t> q((size_t)std::max<int64_t>(n, 1));
        unsigned long long mb = 0;
        if (n) DI_HIP(hipMemcpy(q.data(), dq.p, (size_t)n * 4, hipMemcpyDeviceToHost));
        DI_HIP(hipMemcpy(&mb, dm.p, 8, hipMemcpyDeviceToHost));
        (void)hipSetDevice(prev);
        double m;
        std::memcpy(&m, &mb, 8);
        if (!output_path) {  // max only (find_max_value, quantize.py:17-24; 0 if no term)
            if (max_used) *max_used = m;
            return;
        }
        if (!(max_val > 0.0)) {
            DI_REQUIRE(m > 0.0, DI_EINVAL,
                       "max impact is 0: the reference divides by zero (quantize.py:37)");
            max_val = m;
        }
        if (max_used) *max_used = max_val;
        parallel_for(C, [&](int64_t lo, int64_t hi, int) {
            char num[32];
            for (int64_t c = lo; c < hi; ++c) {
                Part &pc = P[(size_t)c];
                std::string &out = pc.out;
                out.reserve(cut[c + 1] - cut[c]);
                const int32_t *qc = q.data() + off[(size_t)c];
                for (size_t d = 0; d + 1 < pc.cu.size(); ++d) {
                    bool first = true;
                    for (uint32_t i = pc.cu[d]; i < pc.cu[d + 1]; ++i) {
                        if (qc[i] <= 0) continue;  // quantize.py:44
                        if (!first) out += ", ";
                        first = false;
                        out.append(pc.terms[i].data(), pc.terms[i].size());
                        out += ": ";
                        const int len = std::snprintf(num, sizeof num, "%d", qc[i]);
                        out.append(num, (size_t)len);
                    }
                    out += '\n';
                }
            }
        });
        FILE *f = std::fopen(output_path, "wb");
        DI_REQUIRE(f, DI_EIO, "cannot create %s", output_path);
        bool ok = true;
        for (int c = 0; c < C; ++c) {
            const std::string &o = P[(size_t)c].out;
            ok = ok && (o.empty() || std::fwrite(o.data(), 1, o.size(), f) == o.size());
        }
        ok = (std::fclose(f) == 0) && ok;
        DI_REQUIRE(ok, DI_EIO, "short write to %s", output_path);
    });
}
