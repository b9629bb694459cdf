// Native host front end of the scoring path:
//   * BertTokenizer-compatible tokenisation (transformers BertTokenizer: added-token split on
//     the special tokens, BasicTokenizer with do_lower_case — clean text, CJK characters
//     isolated, lower-case + accent stripping, punctuation split — then greedy longest-match
//     WordPiece with "##" continuations, 100-character word limit, [UNK]);
//     replaces MLM_PLL/preprocess.py:9-30 and RescoreBert/preprocess.py:8-55 (tokenizer calls);
//   * vocab.txt loading (one token per line, id = line number, later duplicates win);
//   * the score-JSON writer of util/saving.py:14-16 (json.dump(indent=4, ensure_ascii=False),
//     floats in Python repr).
// Host-only C++17; the Unicode predicates come from unicode_tables.inc (generated from
// Python's unicodedata by tools/gen_unicode_tables.py).  NFC normalisation is the caller's
// (asr_rescoring_amd.frontend applies unicodedata.normalize("NFC") before the call).
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

#include "unicode_tables.inc"

constexpr int kOther = 0, kSpace = 1, kControl = 2, kPunct = 3, kCjk = 4;

int uclass(uint32_t cp) {
    size_t lo = 0, hi = sizeof(kClassRanges) / sizeof(kClassRanges[0]);
    while (lo < hi) {
        const size_t mid = (lo + hi) / 2;
        if (kClassRanges[mid][1] < cp) lo = mid + 1;
        else hi = mid;
    }
    if (lo < sizeof(kClassRanges) / sizeof(kClassRanges[0]) && kClassRanges[lo][0] <= cp) return (int)kClassRanges[lo][2];
    return kOther;
}

template <size_t N, size_t M>
bool map_cp(const uint32_t (&tab)[N][4], const uint32_t (&third)[M][2], uint32_t cp, std::vector<uint32_t>& out) {
    size_t lo = 0, hi = N;
    while (lo < hi) {
        const size_t mid = (lo + hi) / 2;
        if (tab[mid][0] < cp) lo = mid + 1;
        else hi = mid;
    }
    if (lo == N || tab[lo][0] != cp) return false;
    const uint32_t n = tab[lo][1];
    if (n >= 1) out.push_back(tab[lo][2]);
    if (n >= 2) out.push_back(tab[lo][3]);
    if (n >= 3)
        for (size_t k = 0; k < M; ++k)
            if (third[k][0] == cp) out.push_back(third[k][1]);
    return true;
}

void utf8_decode(const char* s, size_t n, std::vector<uint32_t>& out) {
    const unsigned char* p = (const unsigned char*)s;
    size_t i = 0;
    while (i < n) {
        uint32_t c = p[i];
        int len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
        if (len == 0 || i + len > n) {
            out.push_back(0xFFFD);
            ++i;
            continue;
        }
        uint32_t cp = len == 1 ? c : len == 2 ? (c & 0x1F) : len == 3 ? (c & 0x0F) : (c & 0x07);
        bool ok = true;
        for (int k = 1; k < len; ++k) {
            if ((p[i + k] & 0xC0) != 0x80) ok = false;
            cp = (cp << 6) | (p[i + k] & 0x3F);
        }
        out.push_back(ok ? cp : 0xFFFD);
        i += ok ? len : 1;
    }
}

void utf8_append(std::string& s, uint32_t cp) {
    if (cp < 0x80) {
        s += (char)cp;
    } else if (cp < 0x800) {
        s += (char)(0xC0 | (cp >> 6));
        s += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
        s += (char)(0xE0 | (cp >> 12));
        s += (char)(0x80 | ((cp >> 6) & 0x3F));
        s += (char)(0x80 | (cp & 0x3F));
    } else {
        s += (char)(0xF0 | (cp >> 18));
        s += (char)(0x80 | ((cp >> 12) & 0x3F));
        s += (char)(0x80 | ((cp >> 6) & 0x3F));
        s += (char)(0x80 | (cp & 0x3F));
    }
}

std::string to_utf8(const std::vector<uint32_t>& v, size_t b, size_t e) {
    std::string s;
    for (size_t i = b; i < e; ++i) utf8_append(s, v[i]);
    return s;
}

const char* const kSpecial[] = {"[UNK]", "[SEP]", "[PAD]", "[CLS]", "[MASK]"};

struct Vocab {
    std::unordered_map<std::string, int> ids;
    int unk = 0, cls = 101, sep = 102;
    int size = 0;
};

// lower-case then accent-strip one token (BasicTokenizer: token.lower(), _run_strip_accents)
std::vector<uint32_t> normalize_token(const std::vector<uint32_t>& tok) {
    std::vector<uint32_t> low, out;
    for (uint32_t cp : tok)
        if (!map_cp(kLower, kLower_third, cp, low)) low.push_back(cp);
    for (uint32_t cp : low) {
        if (cp >= 0xAC00 && cp <= 0xD7A3) {                 // Hangul syllable: algorithmic NFD
            const uint32_t S = cp - 0xAC00;
            out.push_back(0x1100 + S / 588);
            out.push_back(0x1161 + (S % 588) / 28);
            if (S % 28) out.push_back(0x11A7 + S % 28);
        } else if (!map_cp(kStrip, kStrip_third, cp, out)) {
            out.push_back(cp);
        }
    }
    return out;
}

void wordpiece(const Vocab& v, const std::vector<uint32_t>& w, std::vector<int>& ids) {
    if (w.size() > 100) {
        ids.push_back(v.unk);
        return;
    }
    std::vector<int> sub;
    size_t start = 0;
    while (start < w.size()) {
        size_t end = w.size();
        int cur = -1;
        while (start < end) {
            std::string piece = start > 0 ? "##" : "";
            piece += to_utf8(w, start, end);
            auto it = v.ids.find(piece);
            if (it != v.ids.end()) {
                cur = it->second;
                break;
            }
            --end;
        }
        if (cur < 0) {
            ids.push_back(v.unk);
            return;
        }
        sub.push_back(cur);
        start = end;
    }
    ids.insert(ids.end(), sub.begin(), sub.end());
}

// BasicTokenizer over one segment free of special tokens, then WordPiece
void basic_wordpiece(const Vocab& v, const std::vector<uint32_t>& text, size_t b, size_t e, std::vector<int>& ids) {
    std::vector<uint32_t> t;
    t.reserve(e - b + 16);
    for (size_t i = b; i < e; ++i) {
        const uint32_t cp = text[i];
        if (cp == 0 || cp == 0xFFFD) continue;
        const int k = uclass(cp);
        if (k == kControl) continue;
        // str.split() also breaks on U+2028/U+2029 (Zl/Zp: neither cleaned nor Zs)
        if (k == kSpace || cp == 0x2028 || cp == 0x2029) t.push_back(' ');
        else if (k == kCjk) {
            t.push_back(' ');
            t.push_back(cp);
            t.push_back(' ');
        } else {
            t.push_back(cp);
        }
    }
    size_t i = 0;
    while (i < t.size()) {
        while (i < t.size() && t[i] == ' ') ++i;
        size_t j = i;
        while (j < t.size() && t[j] != ' ') ++j;
        if (j > i) {
            std::vector<uint32_t> tok(t.begin() + i, t.begin() + j);
            const std::vector<uint32_t> nt = normalize_token(tok);
            // punctuation split: every punctuation character is its own word
            size_t s = 0;
            for (size_t q = 0; q <= nt.size(); ++q) {
                const bool end = q == nt.size();
                const bool punct = !end && uclass(nt[q]) == kPunct;
                if (end || punct) {
                    if (q > s) {
                        std::vector<uint32_t> w(nt.begin() + s, nt.begin() + q);
                        // whitespace produced by lower/strip cannot occur (Zs never maps); keep as one word
                        wordpiece(v, w, ids);
                    }
                    if (punct) wordpiece(v, std::vector<uint32_t>{nt[q]}, ids);
                    s = q + 1;
                }
            }
        }
        i = j;
    }
}

void tokenize(const Vocab& v, const char* text, size_t n, bool add_special, std::vector<int>& ids) {
    std::vector<uint32_t> cps;
    utf8_decode(text, n, cps);
    if (add_special) ids.push_back(v.cls);
    // added-token split: exact occurrences of the special tokens are emitted whole
    std::vector<std::vector<uint32_t>> sp;
    for (const char* s : kSpecial) {
        std::vector<uint32_t> c;
        utf8_decode(s, strlen(s), c);
        sp.push_back(c);
    }
    size_t seg = 0, i = 0;
    while (i < cps.size()) {
        int hit = -1;
        for (size_t k = 0; k < sp.size() && hit < 0; ++k)
            if (i + sp[k].size() <= cps.size() && std::equal(sp[k].begin(), sp[k].end(), cps.begin() + i)) hit = (int)k;
        if (hit < 0) {
            ++i;
            continue;
        }
        basic_wordpiece(v, cps, seg, i, ids);
        auto it = v.ids.find(kSpecial[hit]);
        ids.push_back(it != v.ids.end() ? it->second : v.unk);
        i += sp[hit].size();
        seg = i;
    }
    basic_wordpiece(v, cps, seg, cps.size(), ids);
    if (add_special) ids.push_back(v.sep);
}

// ---- JSON (json.dump(indent=4, ensure_ascii=False)) ------------------------------------
void json_string(std::string& o, const char* s) {
    o += '"';
    for (const unsigned char* p = (const unsigned char*)s; *p; ++p) {
        const unsigned char c = *p;
        switch (c) {
            case '"': o += "\\\""; break;
            case '\\': o += "\\\\"; break;
            case '\n': o += "\\n"; break;
            case '\r': o += "\\r"; break;
            case '\t': o += "\\t"; break;
            case '\b': o += "\\b"; break;
            case '\f': o += "\\f"; break;
            default:
                if (c < 0x20) {
                    char b[8];
                    snprintf(b, sizeof(b), "\\u%04x", c);
                    o += b;
                } else {
                    o += (char)c;
                }
        }
    }
    o += '"';
}

// Python float.__repr__: shortest round-trip digits; exponent form when exp < -4 or >= 16
void json_float(std::string& o, double x) {
    if (std::isnan(x)) { o += "NaN"; return; }
    if (std::isinf(x)) { o += x > 0 ? "Infinity" : "-Infinity"; return; }
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof(buf), x, std::chars_format::scientific);
    std::string s(buf, r.ptr);                 // [-]d[.ddd]e(+|-)XX
    std::string sign;
    if (s[0] == '-') { sign = "-"; s = s.substr(1); }
    const size_t epos = s.find('e');
    std::string mant = s.substr(0, epos);
    const int exp = std::stoi(s.substr(epos + 1));
    std::string digits;
    for (char c : mant) if (c != '.') digits += c;
    o += sign;
    if (exp >= -4 && exp < 16) {
        const int nd = (int)digits.size();
        if (exp >= nd - 1) {
            o += digits + std::string(exp - (nd - 1), '0') + ".0";
        } else if (exp >= 0) {
            o += digits.substr(0, exp + 1) + "." + digits.substr(exp + 1);
        } else {
            o += "0." + std::string(-exp - 1, '0') + digits;
        }
    } else {
        o += digits.substr(0, 1);
        if (digits.size() > 1) o += "." + digits.substr(1);
        char e[16];
        snprintf(e, sizeof(e), "e%c%02d", exp < 0 ? '-' : '+', exp < 0 ? -exp : exp);
        o += e;
    }
}

thread_local std::string g_err;

}  // namespace

extern "C" {

void* rs_vocab_load(const char* path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) {
        g_err = std::string("cannot open vocab file ") + path;
        return nullptr;
    }
    Vocab* v = new Vocab();
    std::string line;
    int idx = 0;
    while (std::getline(f, line)) {                 // token = line.rstrip("\n")
        v->ids[line] = idx++;
    }
    v->size = idx;
    auto get = [&](const char* t, int dflt) {
        auto it = v->ids.find(t);
        return it != v->ids.end() ? it->second : dflt;
    };
    v->unk = get("[UNK]", 0);
    v->cls = get("[CLS]", v->unk);
    v->sep = get("[SEP]", v->unk);
    return v;
}

int rs_vocab_size(const void* vocab) { return vocab ? ((const Vocab*)vocab)->size : -1; }

void rs_vocab_free(void* vocab) { delete (Vocab*)vocab; }

// Token ids of n texts (UTF-8, NFC), concatenated; off[h]..off[h+1] per text.  Returns the
// total id count; if it exceeds cap nothing past cap is written and the caller retries with
// a larger buffer (off is always complete).
int64_t rs_tokenize_batch(const void* vocab, const char* const* texts, int n, int add_special,
                          int32_t* ids, int64_t cap, int64_t* off) {
    if (!vocab || n < 0 || (n > 0 && (!texts || !off))) return -1;
    const Vocab& v = *(const Vocab*)vocab;
    // independent texts: contiguous slices on up to 16 host threads, concatenated in order
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int nt = (int)std::min<unsigned>(std::min(hw, 16u), (unsigned)std::max(1, n / 2048));
    std::vector<std::vector<int>> part(nt);
    std::vector<std::vector<int64_t>> plen(nt);
    auto work = [&](int w) {
        const int b = (int)((int64_t)n * w / nt), e = (int)((int64_t)n * (w + 1) / nt);
        std::vector<int> tmp;
        for (int h = b; h < e; ++h) {
            tmp.clear();
            tokenize(v, texts[h], strlen(texts[h]), add_special != 0, tmp);
            part[w].insert(part[w].end(), tmp.begin(), tmp.end());
            plen[w].push_back((int64_t)tmp.size());
        }
    };
    std::vector<std::thread> th;
    for (int w = 1; w < nt; ++w) th.emplace_back(work, w);
    work(0);
    for (auto& t : th) t.join();
    int64_t total = 0;
    int h = 0;
    off[0] = 0;
    for (int w = 0; w < nt; ++w) {
        for (int64_t k = 0; k < (int64_t)part[w].size(); ++k)
            if (ids && total + k < cap) ids[total + k] = part[w][k];
        for (int64_t L : plen[w]) {
            off[h + 1] = off[h] + L;
            ++h;
        }
        total += (int64_t)part[w].size();
    }
    return total;
}

// {utt_id: {hyp_id: score}} for n_utt utterances; hyp_off[u]..hyp_off[u+1] index hyp_ids and
// scores.  Byte-identical to json.dump(obj, f, ensure_ascii=False, indent=4).
int rs_json_write_scores(const char* path, int n_utt, const char* const* utt_ids, const int32_t* hyp_off,
                         const char* const* hyp_ids, const double* scores) {
    std::string o;
    if (n_utt == 0) {
        o = "{}";
    } else {
        o += "{\n";
        for (int u = 0; u < n_utt; ++u) {
            o += "    ";
            json_string(o, utt_ids[u]);
            o += ": ";
            const int b = hyp_off[u], e = hyp_off[u + 1];
            if (b == e) {
                o += "{}";
            } else {
                o += "{\n";
                for (int h = b; h < e; ++h) {
                    o += "        ";
                    json_string(o, hyp_ids[h]);
                    o += ": ";
                    json_float(o, scores[h]);
                    o += h + 1 < e ? ",\n" : "\n";
                }
                o += "    }";
            }
            o += u + 1 < n_utt ? ",\n" : "\n";
        }
        o += "}";
    }
    FILE* f = fopen(path, "wb");
    if (!f) return -1;
    const size_t w = fwrite(o.data(), 1, o.size(), f);
    fclose(f);
    return w == o.size() ? 0 : -1;
}

}  // extern "C"
