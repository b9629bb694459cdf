// Host sanitizer driver for the native front end (csrc/tokenizer.cpp): built with
// -fsanitize=address,undefined by tests/test_host_sanitize.py (ASan/UBSan build of
// the C++ shim).  Exercises every exported entry on adversarial inputs: random and invalid
// UTF-8, control / combining / CJK / punctuation code points, over-long words, empty texts,
// enough texts to take the multi-threaded path, undersized output buffers, and the JSON
// writer with non-finite and extreme doubles and escape-heavy keys.  Exit 0 = no finding
// (any sanitizer report aborts with a non-zero status).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

extern "C" {
void* rs_vocab_load(const char* path);
int rs_vocab_size(const void* vocab);
void rs_vocab_free(void* vocab);
int64_t rs_tokenize_batch(const void* vocab, const char* const* texts, int n, int add_special, int32_t* ids,
                          int64_t cap, int64_t* off);
int rs_json_write_scores(const char* path, int n_utt, const char* const* utt_ids, const int32_t* hyp_off,
                         const char* const* hyp_ids, const double* scores);
}

static void put_utf8(std::string& s, uint32_t cp) {
    if (cp < 0x80) s += (char)cp;
    else if (cp < 0x800) { s += (char)(0xC0 | (cp >> 6)); s += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
        s += (char)(0xE0 | (cp >> 12)); s += (char)(0x80 | ((cp >> 6) & 0x3F)); s += (char)(0x80 | (cp & 0x3F));
    } else {
        s += (char)(0xF0 | (cp >> 18)); s += (char)(0x80 | ((cp >> 12) & 0x3F));
        s += (char)(0x80 | ((cp >> 6) & 0x3F)); s += (char)(0x80 | (cp & 0x3F));
    }
}

int main(int argc, char** argv) {
    const char* dir = argc > 1 ? argv[1] : "/tmp";
    const std::string vpath = std::string(dir) + "/vocab_sanitize.txt";
    {
        FILE* f = fopen(vpath.c_str(), "wb");
        if (!f) return 2;
        const char* toks[] = {"[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]", "the", "##s", "un", "##aff", "##able",
                              "a", "b", "##c", "，", "。", "!", "?", "'", "caf", "##e"};
        for (const char* t : toks) fprintf(f, "%s\n", t);
        std::string cjk;
        for (uint32_t cp = 0x4E00; cp < 0x4E00 + 400; ++cp) { cjk.clear(); put_utf8(cjk, cp); fprintf(f, "%s\n", cjk.c_str()); }
        fclose(f);
    }
    if (rs_vocab_load((std::string(dir) + "/no_such_vocab.txt").c_str()) != nullptr) return 3;
    void* v = rs_vocab_load(vpath.c_str());
    if (!v || rs_vocab_size(v) != 420) return 4;

    std::mt19937_64 rng(12345);
    const uint32_t pool[] = {0x20, 0x09, 0x0A, 0x00AD, 0x0301, 0x0300, 0x2028, 0x3000, 0xFEFF, 0x4E00, 0x4E01, 0x4F60,
                             0x9FFF, 0x3400, 0x20000, 0x2A700, 0xFF01, 0x00E9, 0x00C5, 0x0130, 0x1E9E, 0xFFFD, 0x7F, 0x01};
    std::vector<std::string> texts;
    for (int h = 0; h < 6000; ++h) {
        std::string s;
        const int kind = h % 6;
        const int len = (int)(rng() % (kind == 5 ? 400 : 40));
        for (int i = 0; i < len; ++i) {
            const uint64_t r = rng();
            if (kind == 0) put_utf8(s, pool[r % (sizeof pool / sizeof pool[0])]);
            else if (kind == 1) s += (char)(r & 0xFF ? r & 0xFF : 'x');          // arbitrary (invalid) bytes, no NUL
            else if (kind == 2) s += "unaffable caf\xC3\xA9 the ";
            else if (kind == 3) put_utf8(s, 0x4E00 + (uint32_t)(r % 500));
            else if (kind == 4) s += (char)('a' + r % 3);                       // one long word
            else put_utf8(s, (uint32_t)(r % 0x10FFFF) & ~0x800u);              // any code point
        }
        texts.push_back(s);
    }
    texts.push_back("");
    std::vector<const char*> ptr;
    for (auto& s : texts) ptr.push_back(s.c_str());
    const int n = (int)ptr.size();
    std::vector<int64_t> off(n + 1);
    const int64_t total = rs_tokenize_batch(v, ptr.data(), n, 1, nullptr, 0, off.data());   // size query
    if (total < 2 * n || off[n] != total) return 5;
    for (int h = 0; h < n; ++h)
        if (off[h + 1] - off[h] < 2) return 6;                                 // [CLS] .. [SEP] at least
    std::vector<int32_t> ids(total);
    std::vector<int32_t> small(17);
    if (rs_tokenize_batch(v, ptr.data(), n, 1, small.data(), (int64_t)small.size(), off.data()) != total) return 7;
    if (rs_tokenize_batch(v, ptr.data(), n, 0, ids.data(), total, off.data()) > total) return 8;
    if (rs_tokenize_batch(v, ptr.data(), n, 1, ids.data(), total, off.data()) != total) return 9;
    for (int64_t k = 0; k < total; ++k)
        if (ids[k] < 0 || ids[k] >= 420) return 10;
    if (rs_tokenize_batch(nullptr, ptr.data(), n, 1, ids.data(), total, off.data()) != -1) return 11;
    if (rs_tokenize_batch(v, ptr.data(), 0, 1, ids.data(), total, off.data()) != 0) return 12;

    // JSON writer: escapes, non-ASCII keys, empty utterances, non-finite and extreme values
    std::vector<std::string> utt = {"utt\"1\\", "u\n2\t", "\xE4\xBD\xA0\xE5\xA5\xBD", ""};
    std::vector<std::string> hyp;
    std::vector<double> sc;
    std::vector<int32_t> hoff = {0};
    const double special[] = {0.0, -0.0, 1e-320, 5e-324, 1.7976931348623157e308, -1.5, 0.1, 1e16, 1e-7,
                              123456789.125, NAN, INFINITY, -INFINITY};
    for (size_t u = 0; u < utt.size(); ++u) {
        const int nh = u == 2 ? 0 : 13;
        for (int i = 0; i < nh; ++i) {
            hyp.push_back("hyp_" + std::to_string(i) + (i % 3 == 0 ? "\x01\x1F\"" : ""));
            sc.push_back(special[i % 13] * (u == 3 ? -1.0 : 1.0));
        }
        hoff.push_back((int32_t)hyp.size());
    }
    std::vector<const char*> up, hp;
    for (auto& s : utt) up.push_back(s.c_str());
    for (auto& s : hyp) hp.push_back(s.c_str());
    const std::string jpath = std::string(dir) + "/scores_sanitize.json";
    if (rs_json_write_scores(jpath.c_str(), (int)utt.size(), up.data(), hoff.data(), hp.data(), sc.data()) != 0) return 13;
    if (rs_json_write_scores(jpath.c_str(), 0, nullptr, hoff.data(), nullptr, nullptr) != 0) return 14;
    if (rs_json_write_scores((std::string(dir) + "/no/such/dir/x.json").c_str(), 0, nullptr, hoff.data(), nullptr,
                             nullptr) != -1)
        return 15;
    rs_vocab_free(v);
    rs_vocab_free(nullptr);
    printf("sanitize ok: %d texts, %lld ids\n", n, (long long)total);
    return 0;
}
