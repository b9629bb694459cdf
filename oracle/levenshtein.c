/*
 * ORACLE (test infrastructure only) — C restatement of the edit distance behind
 * ``jiwer.cer`` (third-party, not installed here and unpinned by the reference).
 *
 * Call sites in the reference: rescore.py:40,118 (corpus CER of the argmax hypotheses),
 * RMBR/utility_functions.py:31 (pairwise CER utility), RMBR/main.py:27,95.
 * jiwer >= 3 computes CER as (S + D + I) / (H + S + D) over characters after Strip();
 * S + D + I of a minimal alignment is the unit-cost Levenshtein distance and
 * H + S + D = len(reference).  A list input is a corpus CER: sum of edits / sum of
 * reference lengths.  Here "characters" are int32 symbols (CJK chars = token ids).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may load this.
 * Textbook two-row DP; no bit-parallel tricks (the product kernel has those).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int64_t oracle_levenshtein(const int32_t* a, int32_t na, const int32_t* b, int32_t nb) {
    if (na == 0) return nb;
    if (nb == 0) return na;
    int64_t* prev = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nb + 1));
    int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nb + 1));
    for (int32_t j = 0; j <= nb; ++j) prev[j] = j;
    for (int32_t i = 1; i <= na; ++i) {
        cur[0] = i;
        for (int32_t j = 1; j <= nb; ++j) {
            int64_t sub = prev[j - 1] + (a[i - 1] != b[j - 1]);
            int64_t del = prev[j] + 1;
            int64_t ins = cur[j - 1] + 1;
            int64_t m = sub < del ? sub : del;
            cur[j] = m < ins ? m : ins;
        }
        int64_t* t = prev; prev = cur; cur = t;
    }
    int64_t d = prev[nb];
    free(prev);
    free(cur);
    return d;
}

/* Pairwise distance matrices for ragged strings grouped by utterance.
 * str_off[s]..str_off[s+1] delimits string s in chars; utt_off[u]..utt_off[u+1]
 * delimits the strings of utterance u; out is the concatenation of the per-utterance
 * n_u x n_u matrices, row-major, out[(i, j)] = ed(string_i, string_j). */
void oracle_pairwise(const int32_t* chars, const int32_t* str_off, const int32_t* utt_off,
                     int32_t n_utt, int64_t* out) {
    int64_t o = 0;
    for (int32_t u = 0; u < n_utt; ++u) {
        int32_t s0 = utt_off[u], n = utt_off[u + 1] - utt_off[u];
        for (int32_t i = 0; i < n; ++i)
            for (int32_t j = 0; j < n; ++j) {
                const int32_t* a = chars + str_off[s0 + i];
                const int32_t* b = chars + str_off[s0 + j];
                out[o++] = oracle_levenshtein(a, str_off[s0 + i + 1] - str_off[s0 + i],
                                              b, str_off[s0 + j + 1] - str_off[s0 + j]);
            }
    }
}
