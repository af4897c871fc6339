// text_index.cpp -- native builder of the reference's on-disk index files.
//
// Replaces InvertedIndexCreator (reference src/deep_impact/inverted_index/
// create.py:12-55) reading the collection through DeepImpactCollection
// (src/deep_impact/indexing/deep_impact_collection.py:6-33); output is
// byte-identical: vocab.txt, inverted_index.idx, inverted_index.dat.
#include <algorithm>
#include <cstdio>
#include <fstream>
#include <string>
#include <string_view>
#include <unordered_map>
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
    std::vector<int64_t> val;            // int(float(text))
    std::vector<int64_t> cu;             // per doc
};

// DeepImpactCollection.__getitem__: line.strip(); '' -> {}; else
// {term: float(v) for term, v in (p.split(': ') for p in s.split(', '))}
// (a dict: a repeated term keeps its first position and its last value).
void parse_collection(std::string_view buf, Parsed &P) {
    P.cu.push_back(0);
    std::vector<std::string_view> pairs, tv;
    std::unordered_map<std::string_view, size_t> seen;
    int64_t line_no = 0;
    py::for_each_line(buf, [&](std::string_view line) {
        ++line_no;
        std::string_view s = py::strip(line);
        if (!py::strip(s).empty()) {
            py::split(s, ", ", pairs);
            seen.clear();
            for (auto pr : pairs) {
                py::split(pr, ": ", tv);
                DI_REQUIRE(tv.size() == 2, DI_EFORMAT,
                           "line %lld: '%.*s' does not split into term and value (reference "
                           "raises ValueError)",
                           (long long)line_no, (int)std::min<size_t>(pr.size(), 200), pr.data());
                double v;
                DI_REQUIRE(py::parse_float(tv[1], &v), DI_EFORMAT,
                           "line %lld: could not convert '%.*s' to float", (long long)line_no,
                           (int)std::min<size_t>(tv[1].size(), 64), tv[1].data());
                DI_REQUIRE(!std::isnan(v) && !std::isinf(v), DI_EFORMAT,
                           "line %lld: int() of a non-finite value", (long long)line_no);
                int64_t iv = (int64_t)std::trunc(v);
                auto it = seen.find(tv[0]);
                if (it != seen.end()) {
                    P.val[it->second] = iv;  // dict: last value wins
                } else {
                    seen.emplace(tv[0], P.term.size());
                    P.term.push_back(tv[0]);
                    P.val.push_back(iv);
                }
            }
        }
        P.cu.push_back((int64_t)P.term.size());
    });
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
        std::string buf = read_file(collection_path);
        Parsed P;
        parse_collection(buf, P);
        const int64_t n_docs = (int64_t)P.cu.size() - 1;
        DI_REQUIRE(n_docs <= 0xFFFFFFFFll, DI_ERANGE, "more than 2^32 documents");
        // vocab: sorted(set(terms)) -- code-point order == UTF-8 byte order
        std::unordered_map<std::string_view, uint32_t> ids;
        ids.reserve(P.term.size() / 8 + 16);
        std::vector<std::string_view> vocab;
        for (auto t : P.term)
            if (ids.emplace(t, 0).second) vocab.push_back(t);
        std::sort(vocab.begin(), vocab.end());
        for (size_t i = 0; i < vocab.size(); ++i) ids[vocab[i]] = (uint32_t)i;
        const size_t V = vocab.size();
        // postings: per term, docs in order; stable by value descending
        for (auto v : P.val)
            DI_REQUIRE(v >= 0 && v <= 255, DI_EFORMAT,
                       "value %lld does not fit the 1-byte impact record (struct.error in "
                       "the reference)",
                       (long long)v);
        // bucket by term (doc order), then a stable value-descending sort per term
        std::vector<int64_t> toff(V + 1, 0);
        std::vector<uint32_t> tid(P.term.size());
        for (size_t i = 0; i < P.term.size(); ++i) {
            tid[i] = ids[P.term[i]];
            toff[tid[i] + 1]++;
        }
        for (size_t t = 0; t < V; ++t) toff[t + 1] += toff[t];
        std::vector<uint32_t> bdoc(P.term.size());
        std::vector<uint8_t> bval(P.term.size());
        {
            std::vector<int64_t> cur(toff.begin(), toff.end() - 1);
            for (int64_t d = 0; d < n_docs; ++d)
                for (int64_t i = P.cu[d]; i < P.cu[d + 1]; ++i) {
                    int64_t pos = cur[tid[i]]++;
                    bdoc[pos] = (uint32_t)d;
                    bval[pos] = (uint8_t)P.val[i];
                }
        }
        std::vector<unsigned char> dat(P.term.size() * 5);
        std::vector<int64_t> vc(257);
        for (size_t t = 0; t < V; ++t) {
            const int64_t a = toff[t], b = toff[t + 1];
            std::fill(vc.begin(), vc.end(), 0);
            for (int64_t i = a; i < b; ++i) vc[(size_t)(255 - bval[i]) + 1]++;
            for (int c = 0; c < 256; ++c) vc[c + 1] += vc[c];
            for (int64_t i = a; i < b; ++i) {
                int64_t pos = a + vc[(size_t)(255 - bval[i])]++;
                std::memcpy(&dat[(size_t)pos * 5], &bdoc[i], 4);
                dat[(size_t)pos * 5 + 4] = bval[i];
            }
        }
        std::vector<uint64_t> idx(V * 2);
        for (size_t t = 0; t < V; ++t) {
            idx[2 * t] = (uint64_t)toff[t] * 5;
            idx[2 * t + 1] = (uint64_t)toff[t + 1] * 5;
        }
        std::string vtxt;
        vtxt.reserve(V * 8);
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
