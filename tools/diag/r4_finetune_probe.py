"""Round-4 probe: how many MLM fine-tuning steps on the synthetic set's reference sentences make
the bench's LM informative (best fusion weight > 0, reranked CER < AM-only CER)?
Usage: python tools/diag/r4_finetune_probe.py [utts] [lr] [batch] [checkpoints...]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import data as D, rerank  # noqa: E402
from asr_rescoring_amd.scorer import PLLScorer  # noqa: E402
from asr_rescoring_amd.train import MLMTrainer, pad_rows  # noqa: E402
from asr_rescoring_amd.weights import BERT_BASE, make_weights  # noqa: E402


def main():
    U = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    lr = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-4
    bs = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    cps = [int(x) for x in sys.argv[4:]] or [0, 100, 200, 400, 800]
    nb = D.synthetic_nbest(U, 50, seed=1, hard=True)
    w = make_weights(BERT_BASE, seed=1234)
    seqs, labels = [], []
    for r in nb.refs:
        h = [101] + [int(x) for x in r] + [102]
        for p in range(1, len(h) - 1):
            row = list(h)
            row[p] = 103
            seqs.append(row)
            labels.append(h)
    tr = MLMTrainer(w, BERT_BASE, device=0, lr=lr, hidden_dropout=0.0, attn_dropout=0.0)
    rng = np.random.Generator(np.random.PCG64(0))
    order = np.empty(0, np.int64)
    done = 0
    t_train = 0.0
    for cp in cps:
        t0 = time.perf_counter()
        while done < cp:
            if len(order) < bs:
                order = np.concatenate([order, rng.permutation(len(seqs))])
            sel, order = order[:bs], order[bs:]
            ids, off, lab, klen = pad_rows([seqs[i] for i in sel], [labels[i] for i in sel])
            loss = tr.step(ids, off, lab, klen)
            done += 1
        torch.cuda.synchronize()
        t_train += time.perf_counter() - t0
        sd = tr.state_dict()
        sc = PLLScorer(sd, BERT_BASE, device=0, max_rows=262144)
        lm = sc.score(nb)
        sc.close()
        bw, bcer, arg, cers = rerank.find_best_weight(nb, lm, n_best=50, device=0)
        print(f"steps {cp} (lr {lr}, batch {bs}, train {t_train:.1f}s, last loss {loss if cp else float('nan'):.4f}): "
              f"best_weight {bw:.2f} cer {bcer:.5f} am_only {cers[0]:.5f} cer@w=0.5 {cers[50]:.5f}", flush=True)
    tr.close()


if __name__ == "__main__":
    main()
