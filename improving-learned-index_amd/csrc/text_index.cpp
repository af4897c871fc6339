// text_index.cpp -- native builder of the reference's on-disk index files.
//
// Replaces InvertedIndexCreator (reference src/deep_impact/inverted_index/
// create.py:12-55) reading the collection through DeepImpactCollection
// (src/deep_impact/indexing/deep_impact_collection.py:6-33); output is
// byte-identical: vocab.txt, inverted_index.idx, inverted_index.dat.
//
// Every pass runs on host_threads() threads (the per-term counting passes on as many
// as fit a memory budget): the collection is cut into ranges of
// whole lines (parsed in parallel, doc ids = global line numbers), the vocabulary is
// the union of per-thread term sets merged by hash partition and sorted, the postings
// are bucketed by term with per-thread write offsets (doc order inside a term), then
// stable-sorted by value descending per term.  The output does not depend on the
// thread count.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <string>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "di_common.h"
#include "pytext.h"

namespace {

using namespace di;

std::string read_file(const char *path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    DI_REQUIRE(f, DI_EIO, "cannot open %s", path);
    std::string s((size_t)f.tellg(), '\0');
    f.seekg(0);
    f.read(s.data(), (std::streamsize)s.size());
    DI_REQUIRE(f || s.empty(), DI_EIO, "cannot read %s", path);
    return s;
}

struct Parsed {
    std::vector<std::string_view> term;  // per posting, doc order
    std::vector<uint16_t> val;           // int(float(text)); 256: outside the 1-byte record
    std::vector<uint32_t> cu;            // per doc (local)
};

// DeepImpactCollection.__getitem__: line.strip(); '' -> {}; else
// {term: float(v) for term, v in (p.split(': ') for p in s.split(', '))}
// (a dict: a repeated term keeps its first position and its last value).  A line is
// taken as parsed; then the sorted hashes of its terms show whether any term repeats
// (rare), and only then is the dict rule applied.
inline uint64_t fnv1a(std::string_view x) {
    uint64_t h = 0xCBF29CE484222325ull;
    for (unsigned char c : x) h = (h ^ c) * 0x100000001B3ull;
    return h;
}

void parse_collection(std::string_view buf, Parsed &P, int64_t *ln) {
    P.cu.push_back(0);
    std::vector<std::string_view> pairs, tv;
    std::vector<std::pair<uint64_t, uint32_t>> hs;
    py::for_each_line(buf, [&](std::string_view line) {
        ++*ln;
        std::string_view s = py::strip(line);
        if (!py::strip(s).empty()) {
            py::split(s, ", ", pairs);
            const size_t first = P.term.size();
            for (auto pr : pairs) {
                py::split(pr, ": ", tv);
                DI_REQUIRE(tv.size() == 2, DI_EFORMAT,
                           "'%.*s' does not split into term and value (reference raises "
                           "ValueError)",
                           (int)std::min<size_t>(pr.size(), 200), pr.data());
                double v;
                DI_REQUIRE(py::parse_float(tv[1], &v), DI_EFORMAT,
                           "could not convert '%.*s' to float",
                           (int)std::min<size_t>(tv[1].size(), 64), tv[1].data());
                DI_REQUIRE(!std::isnan(v) && !std::isinf(v), DI_EFORMAT,
                           "int() of a non-finite value");
                const double t = std::trunc(v);
                // (checked on the dict's final values below: a later value of a repeated
                // term replaces an earlier one)
                P.term.push_back(tv[0]);
                P.val.push_back(t >= 0.0 && t <= 255.0 ? (uint16_t)t : (uint16_t)256);
            }
            const size_t n = P.term.size() - first;
            if (n > 1) {
                hs.resize(n);
                for (size_t i = 0; i < n; ++i) hs[i] = {fnv1a(P.term[first + i]), (uint32_t)i};
                std::sort(hs.begin(), hs.end());
                // any equal hash (a repeat, or a collision of two different terms) takes
                // the exact path: with a collision, sorted neighbours need not be the
                // repeat itself
                bool dup = false;
                for (size_t i = 1; i < n && !dup; ++i) dup = hs[i].first == hs[i - 1].first;
                if (dup) {  // the dict: first slot, last value
                    std::unordered_map<std::string_view, size_t> seen;
                    size_t o = first;
                    for (size_t i = first; i < first + n; ++i) {
                        auto it = seen.find(P.term[i]);
                        if (it != seen.end()) {
                            P.val[it->second] = P.val[i];
                        } else {
                            seen.emplace(P.term[i], o);
                            P.term[o] = P.term[i];
                            P.val[o] = P.val[i];
                            ++o;
                        }
                    }
                    P.term.resize(o);
                    P.val.resize(o);
                }
            }
        }
        P.cu.push_back((uint32_t)P.term.size());
    });
    for (size_t d = 0; d + 1 < P.cu.size(); ++d)
        for (uint32_t i = P.cu[d]; i < P.cu[d + 1]; ++i)
            if (P.val[i] > 255) {
                *ln = (int64_t)d + 1;  // (the line of the offending value)
                DI_REQUIRE(false, DI_EFORMAT,
                           "a value does not fit the 1-byte impact record (struct.error in "
                           "the reference)");
            }
}

// Threads for the per-term count arrays (V u32 counters per thread): at most
// host_threads(), and no more than fit kCountBudget bytes together (V = 17.6 M terms
// is 70 MB per thread).
constexpr size_t kCountBudget = size_t(1) << 30;
int count_threads(size_t V, int T) {
    const size_t per = std::max<size_t>(V, 1) * sizeof(uint32_t);
    return (int)std::max<size_t>(1, std::min<size_t>((size_t)T, kCountBudget / per));
}

void write_all(const std::string &path, const void *data, size_t n) {
    FILE *f = std::fopen(path.c_str(), "wb");
    DI_REQUIRE(f, DI_EIO, "cannot create %s", path.c_str());
    size_t w = n ? std::fwrite(data, 1, n, f) : 0;
    int rc = std::fclose(f);
    DI_REQUIRE(w == n && rc == 0, DI_EIO, "short write to %s", path.c_str());
}

}  // namespace

extern "C" int di_build_reference_index(const char *collection_path, const char *out_dir) {
    return guard([&] {
        DI_REQUIRE(collection_path && out_dir, DI_EINVAL, "null argument");
        const std::string buf = read_file(collection_path);
        const int T = host_threads();
        // 1. parse ranges of whole lines in parallel
        const std::vector<size_t> cut = py::line_chunks(buf, 8 * T);
        const int C = (int)cut.size() - 1;
        std::vector<Parsed> P((size_t)std::max(C, 1));
        parallel_chunks(C, [&](int64_t c, int) {
            int64_t ln = 0;
            with_line_context(
                [&] {
                    parse_collection(std::string_view(buf).substr(cut[c], cut[c + 1] - cut[c]),
                                     P[(size_t)c], &ln);
                },
                [&] { return py::count_lines(std::string_view(buf).substr(0, cut[c])) + ln; });
        });
        std::vector<int64_t> doc0((size_t)C + 1, 0), occ0((size_t)C + 1, 0);
        for (int c = 0; c < C; ++c) {
            doc0[(size_t)c + 1] = doc0[(size_t)c] + (int64_t)P[(size_t)c].cu.size() - 1;
            occ0[(size_t)c + 1] = occ0[(size_t)c] + (int64_t)P[(size_t)c].term.size();
        }
        const int64_t n_docs = doc0[(size_t)C], n_occ = occ0[(size_t)C];
        DI_REQUIRE(n_docs <= 0xFFFFFFFFll, DI_ERANGE, "more than 2^32 documents");
        // 2. vocabulary: sorted(set(terms)) -- code-point order == UTF-8 byte order.
        // Per-thread sets over contiguous chunk ranges, each dealt once into T hash
        // partitions; partition p then merges its T buckets (total work ~ the sets'
        // sizes, not T times them).
        const std::hash<std::string_view> H;
        std::vector<std::vector<std::vector<std::string_view>>> bucket(
            (size_t)T, std::vector<std::vector<std::string_view>>((size_t)T));
        parallel_for_threads(C, T, [&](int64_t lo, int64_t hi, int t) {
            std::unordered_set<std::string_view> st;
            for (int64_t c = lo; c < hi; ++c)
                for (auto x : P[(size_t)c].term) st.insert(x);
            auto &b = bucket[(size_t)t];
            for (auto x : st) b[H(x) % (size_t)T].push_back(x);
        });
        std::vector<std::vector<std::string_view>> part((size_t)T);
        parallel_for_threads(T, T, [&](int64_t lo, int64_t hi, int) {
            for (int64_t p = lo; p < hi; ++p) {
                size_t m = 0;
                for (auto &b : bucket) m += b[(size_t)p].size();
                std::unordered_set<std::string_view> u;
                u.reserve(m);
                for (auto &b : bucket) {
                    for (auto x : b[(size_t)p]) u.insert(x);
                    std::vector<std::string_view>().swap(b[(size_t)p]);
                }
                part[(size_t)p].assign(u.begin(), u.end());
            }
        });
        decltype(bucket)().swap(bucket);
        std::vector<std::string_view> vocab;
        for (auto &pp : part) vocab.insert(vocab.end(), pp.begin(), pp.end());
        std::sort(vocab.begin(), vocab.end());
        const size_t V = vocab.size();
        DI_REQUIRE(V < 0xFFFFFFFFull, DI_ERANGE, "more than 2^32 terms");
        // id lookup: per-partition maps (built in parallel, read-only after)
        std::vector<std::unordered_map<std::string_view, uint32_t>> idmap((size_t)T);
        parallel_for_threads(T, T, [&](int64_t lo, int64_t hi, int) {
            for (int64_t p = lo; p < hi; ++p) idmap[(size_t)p].reserve(part[(size_t)p].size());
        });
        parallel_for_threads(T, T, [&](int64_t lo, int64_t hi, int) {
            for (int64_t p = lo; p < hi; ++p)
                for (auto x : part[(size_t)p]) idmap[(size_t)p].emplace(x, 0u);
        });
        parallel_for((int64_t)V, [&](int64_t lo, int64_t hi, int) {
            for (int64_t i = lo; i < hi; ++i) {
                auto x = vocab[(size_t)i];
                idmap[H(x) % (size_t)T].find(x)->second = (uint32_t)i;  // (own slot: no race)
            }
        });
        // 3. term id of every occurrence; per-thread counts per term (TC threads: the
        // count arrays are V words each, kept within kCountBudget together)
        const int TC = count_threads(V, T);
        std::vector<uint32_t> tid((size_t)std::max<int64_t>(n_occ, 1));
        std::vector<std::vector<uint32_t>> tcnt((size_t)TC);
        parallel_for_threads(C, TC, [&](int64_t lo, int64_t hi, int t) {
            auto &cnt = tcnt[(size_t)t];
            cnt.assign(V, 0);
            for (int64_t c = lo; c < hi; ++c) {
                const auto &pc = P[(size_t)c];
                for (size_t i = 0; i < pc.term.size(); ++i) {
                    auto x = pc.term[i];
                    const uint32_t id = idmap[H(x) % (size_t)T].find(x)->second;
                    tid[(size_t)occ0[(size_t)c] + i] = id;
                    cnt[id]++;
                }
            }
        });
        std::vector<std::unordered_map<std::string_view, uint32_t>>().swap(idmap);
        // toff[t] and each thread's write offset per term (doc order inside a term:
        // threads own ascending doc ranges)
        std::vector<int64_t> toff(V + 1, 0);
        std::vector<std::vector<uint32_t>> &tpos = tcnt;  // counts -> offsets in place
        for (size_t t = 0; t < V; ++t) {
            int64_t run = toff[t];
            for (int th = 0; th < TC; ++th) {
                auto &v = tpos[(size_t)th];
                if (v.empty()) continue;
                const uint32_t c = v[t];
                v[t] = (uint32_t)(run - toff[t]);  // offset within the term
                run += c;
            }
            toff[t + 1] = run;
        }
        std::vector<uint32_t> bdoc((size_t)std::max<int64_t>(n_occ, 1));
        std::vector<uint8_t> bval((size_t)std::max<int64_t>(n_occ, 1));
        // (same TC threads and chunk ranges as the counting pass: thread t's offsets)
        parallel_for_threads(C, TC, [&](int64_t lo, int64_t hi, int t) {
            auto &off = tpos[(size_t)t];
            for (int64_t c = lo; c < hi; ++c) {
                const auto &pc = P[(size_t)c];
                for (size_t d = 0; d + 1 < pc.cu.size(); ++d) {
                    const uint32_t doc = (uint32_t)(doc0[(size_t)c] + (int64_t)d);
                    for (uint32_t i = pc.cu[d]; i < pc.cu[d + 1]; ++i) {
                        const uint32_t id = tid[(size_t)occ0[(size_t)c] + i];
                        const int64_t pos = toff[id] + off[id]++;
                        bdoc[(size_t)pos] = doc;
                        bval[(size_t)pos] = (uint8_t)pc.val[i];
                    }
                }
            }
        });
        std::vector<std::vector<uint32_t>>().swap(tcnt);
        std::vector<uint32_t>().swap(tid);
        // 4. per term: stable sort by value descending (create.py:41) into the records
        std::vector<unsigned char> dat((size_t)n_occ * 5);
        parallel_for((int64_t)V, [&](int64_t lo, int64_t hi, int) {
            std::vector<int64_t> vc(257);
            std::vector<uint32_t> ord;
            for (int64_t t = lo; t < hi; ++t) {
                const int64_t a = toff[(size_t)t], b = toff[(size_t)t + 1];
                if (b - a <= 32) {  // short list: stable insertion order by value desc
                    ord.resize((size_t)(b - a));
                    for (int64_t i = 0; i < b - a; ++i) {
                        int64_t j = i;
                        while (j > 0 && bval[(size_t)(a + ord[(size_t)j - 1])] < bval[(size_t)(a + i)]) {
                            ord[(size_t)j] = ord[(size_t)j - 1];
                            --j;
                        }
                        ord[(size_t)j] = (uint32_t)i;
                    }
                    for (int64_t i = 0; i < b - a; ++i) {
                        const int64_t s = a + ord[(size_t)i];
                        std::memcpy(&dat[(size_t)(a + i) * 5], &bdoc[(size_t)s], 4);
                        dat[(size_t)(a + i) * 5 + 4] = bval[(size_t)s];
                    }
                    continue;
                }
                std::fill(vc.begin(), vc.end(), 0);
                for (int64_t i = a; i < b; ++i) vc[(size_t)(255 - bval[(size_t)i]) + 1]++;
                for (int c = 0; c < 256; ++c) vc[(size_t)c + 1] += vc[(size_t)c];
                for (int64_t i = a; i < b; ++i) {
                    const int64_t pos = a + vc[(size_t)(255 - bval[(size_t)i])]++;
                    std::memcpy(&dat[(size_t)pos * 5], &bdoc[(size_t)i], 4);
                    dat[(size_t)pos * 5 + 4] = bval[(size_t)i];
                }
            }
        });
        std::vector<uint64_t> idx(V * 2);
        for (size_t t = 0; t < V; ++t) {
            idx[2 * t] = (uint64_t)toff[t] * 5;
            idx[2 * t + 1] = (uint64_t)toff[t + 1] * 5;
        }
        std::string vtxt;
        size_t vbytes = 0;
        for (auto t : vocab) vbytes += t.size() + 1;
        vtxt.reserve(vbytes);
        for (auto t : vocab) {
            vtxt.append(t.data(), t.size());
            vtxt += '\n';
        }
        std::string od(out_dir);
        write_all(od + "/vocab.txt", vtxt.data(), vtxt.size());
        write_all(od + "/inverted_index.dat", dat.data(), dat.size());
        write_all(od + "/inverted_index.idx", idx.data(), idx.size() * 8);
    });
}
