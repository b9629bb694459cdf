"""BERTScore oracle (CPU): the embedding step against transformers.BertModel (the class
bert_score loads, truncated to num_layers), and properties of the greedy matching that
bert_score's definition implies (parity of the matching itself: unpinned, bert_score absent)."""
import numpy as np
import pytest
import torch

from asr_rescoring_amd.weights import BERT_TINY, make_weights
from oracle import bertscore_ref as B

transformers = pytest.importorskip("transformers")


@pytest.fixture(scope="module")
def tiny():
    w = make_weights(BERT_TINY, seed=11)
    return w, B.truncated_model(w, BERT_TINY, 1)


def _sent(rng, L):
    return [101] + rng.integers(106, BERT_TINY.vocab, size=L).tolist() + [102]


def test_embedding_matches_transformers_bertmodel(tiny):
    w, model = tiny
    cfg = transformers.BertConfig(vocab_size=BERT_TINY.vocab, hidden_size=BERT_TINY.hidden, num_hidden_layers=1,
                                  num_attention_heads=BERT_TINY.heads, intermediate_size=BERT_TINY.intermediate,
                                  max_position_embeddings=BERT_TINY.max_pos, layer_norm_eps=BERT_TINY.ln_eps,
                                  hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    ref = transformers.BertModel(cfg, add_pooling_layer=False).eval()
    sd = {k[len("bert."):]: torch.from_numpy(np.ascontiguousarray(v)) for k, v in w.items()
          if k.startswith("bert.") and (not k.startswith("bert.encoder.layer.") or k.split(".")[3] == "0")}
    missing, unexpected = ref.load_state_dict(sd, strict=False)
    assert not [m for m in missing if "position_ids" not in m], missing
    rng = np.random.default_rng(0)
    sents = [_sent(rng, L) for L in (0, 3, 17, 40)]
    embs = B.embed_sentences(model, sents)
    for s, e in zip(sents, embs):
        with torch.no_grad():
            want = ref(torch.tensor([s]), attention_mask=torch.ones(1, len(s), dtype=torch.long)).last_hidden_state[0]
        assert torch.allclose(e, want, atol=2e-5, rtol=1e-5)


def test_greedy_matching_properties(tiny):
    _, model = tiny
    rng = np.random.default_rng(1)
    a, b, c = _sent(rng, 9), _sent(rng, 14), [101, 102]
    P, R, F = B.bert_score(model, [a, a, b, c, a], [a, b, a, a, c])
    assert np.allclose([P[0], R[0], F[0]], 1.0, atol=1e-6)         # identical sentences
    assert abs(P[1] - R[2]) < 1e-6 and abs(R[1] - P[2]) < 1e-6       # P(a|b) = R(b|a)
    assert P[3] == R[3] == F[3] == 0.0 and P[4] == R[4] == F[4] == 0.0  # empty side
    assert abs(F[1] - 2 * P[1] * R[1] / (P[1] + R[1])) < 1e-6


def test_mbr_on_utility_matrix_order():
    m = np.array([[0, .5, .25], [.75, 0, .5], [.5, .5, 0]], np.float32)
    am, sc = B.mbr_decode(3, [m])
    assert sc[0].tolist() == [0.75, 1.25, 1.0] and am[0] == 1
