"""End-to-end C1 plumbing through the CLI drivers (reference entry points) on the GPU:
hyps_text -> mlm_pll (PLL JSON) -> rescore (best weight, dev/test CER) -> rmbr (CER utility)."""
import json
import os

import numpy as np
import pytest
import yaml

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c1(golden_dir, tmp_path_factory):
    g = json.load(open(os.path.join(golden_dir, "c1_plumbing.json"), encoding="utf-8"))
    d = tmp_path_factory.mktemp("c1")
    for name in ("hyps_text", "ref_text", "hyps_score"):
        json.dump(g[name], open(d / f"{name}.json", "w", encoding="utf-8"), ensure_ascii=False)
    # vocab.txt reproducing the fixture's char ids (106 + index in the sorted charset)
    special = {0: "[PAD]", 100: "[UNK]", 101: "[CLS]", 102: "[SEP]", 103: "[MASK]"}
    lines = [special.get(i, f"[unused{i}]") for i in range(106)] + list(g["charset"])
    (d / "vocab.txt").write_text("\n".join(lines) + "\n", encoding="utf-8")
    return g, d


def _cfg(d, name, obj):
    p = d / name
    p.write_text(yaml.safe_dump(obj, allow_unicode=True), encoding="utf-8")
    return str(p)


def test_cli_c1_pipeline(c1):
    from asr_rescoring_amd import cli
    g, d = c1
    out = str(d) + "/"
    assert cli.main(["mlm_pll", "--config", _cfg(d, "score.yaml", {
        "task": "scoring", "seed": 10, "device": "cuda:0", "random_init_seed": 1234,
        "train_hyps_text_path": str(d / "hyps_text.json"), "output_path": out,
        "model": {"bert": "bert-base-chinese", "vocab": str(d / "vocab.txt")}})]) == 0
    lm = json.load(open(out + "train_lm.json", encoding="utf-8"))
    assert list(lm) == g["utt_ids"]
    got = np.array([v for u in lm for v in lm[u].values()])
    ref = np.array([v for u in g["lm"] for v in g["lm"][u].values()])
    assert (np.abs(got - ref) / np.abs(ref)).max() < 1e-3

    paths = {f"{s}_{k}_path": str(d / f) for s in ("dev", "test")
             for k, f in (("am", "hyps_score.json"), ("hyps_text", "hyps_text.json"), ("ref_text", "ref_text.json"))}
    paths.update({"dev_lm_path": out + "train_lm.json", "test_lm_path": out + "train_lm.json"})
    res = cli.rescore(cli.ArgParser().parse(["--config", _cfg(d, "rescore.yaml", {
        **paths, "n_best": 10, "output_path": str(d / "rescore_out")})]))
    assert res["best_weight"] == g["best_weight"] and res["dev_cer"] == g["best_cer"]
    log = (d / "rescore_out" / "rescore.log").read_text()
    assert "best_weight: " in log and "dev cer: " in log and "test cer: " in log

    res2 = cli.rmbr(cli.ArgParser().parse(["--config", _cfg(d, "CER.yaml", {
        "device": "cuda:0", "utility_function": "cer",
        "dev_feature": ["ref_text", "hyps_text"], "test_feature": ["ref_text", "hyps_text"],
        "dev_feature_path": [str(d / "ref_text.json"), str(d / "hyps_text.json")],
        "test_feature_path": [str(d / "ref_text.json"), str(d / "hyps_text.json")],
        "dev_output_format": str(d / "hyps_score.json"), "test_output_format": str(d / "hyps_score.json"),
        "output_path": str(d / "mbr_out"), "max_utt": 99999999, "n_best": 10})]))
    # oracle restatement of RMBR on the same texts
    from oracle import rescore_ref as R
    hyps = [[[ord(c) for c in t.strip()] for t in g["hyps_text"][u].values()] for u in g["utt_ids"]]
    refs = [[ord(c) for c in g["ref_text"][u].strip()] for u in g["utt_ids"]]
    bc, bl, _ = R.find_best_length(10, refs, hyps)
    assert res2["best_length"] == bl and res2["best_cer"] == bc
    mbr = json.load(open(d / "mbr_out" / "test_MBR.json", encoding="utf-8"))
    assert list(mbr) == g["utt_ids"]


def test_cli_rmbr_bertscore(c1):
    """RMBR with utility_function: bertscore (8-layer bert-base, seeded weights) on the C1
    texts: dev_MBR.json scores at the chosen length equal the oracle's bert_score MBR."""
    from asr_rescoring_amd import cli
    from asr_rescoring_amd.frontend import NativeTokenizer
    from asr_rescoring_amd.weights import BERT_BASE, make_weights
    from oracle import bertscore_ref as B
    g, d = c1
    res = cli.rmbr(cli.ArgParser().parse(["--config", _cfg(d, "BertScore.yaml", {
        "device": "cuda:0", "utility_function": "bertscore", "random_init_seed": 1234,
        "model": {"bert": "bert-base-chinese", "vocab": str(d / "vocab.txt")},
        "dev_feature": ["ref_text", "hyps_text"], "test_feature": ["ref_text", "hyps_text"],
        "dev_feature_path": [str(d / "ref_text.json"), str(d / "hyps_text.json")],
        "test_feature_path": [str(d / "ref_text.json"), str(d / "hyps_text.json")],
        "dev_output_format": str(d / "hyps_score.json"), "test_output_format": str(d / "hyps_score.json"),
        "output_path": str(d / "mbr_bs_out"), "max_utt": 99999999, "n_best": 10})]))
    assert 2 <= res["best_length"] <= 10 and 0.0 <= res["best_cer"] <= 1.0
    tok = NativeTokenizer(str(d / "vocab.txt"))
    utts = [[[101] + tok.encode(t) + [102] for t in list(g["hyps_text"][u].values())[:10]] for u in g["utt_ids"]]
    model = B.truncated_model(make_weights(BERT_BASE, seed=1234), BERT_BASE, 8)
    k = res["best_length"]
    _, want = B.mbr_decode(k, B.utility_matrices(model, utts, "R"))
    mbr = json.load(open(d / "mbr_bs_out" / "dev_MBR.json", encoding="utf-8"))
    got = np.array([list(mbr[u].values())[:k] for u in g["utt_ids"]], np.float32)
    assert np.allclose(got, want, rtol=1e-3, atol=1e-5)


def test_cli_rescorebert_train_then_score(c1):
    """rescorebert_train with the reference's MD_MWER_train.yaml layout (method,
    md_loss_weight, epoch, batch_size in utterances, hyps_token_ids / mlm_pll_score /
    hyps_am_score / hyps_cer features) on the C1 texts (teacher = the golden lm JSON):
    checkpoint_{n}.pth + loss.json per epoch; resuming at epoch 2 from checkpoint_1.pth
    reproduces the straight run bitwise (AdamW is rebuilt every epoch, as in the reference);
    the checkpoint then feeds rescorebert scoring."""
    import torch
    from asr_rescoring_amd import cli
    g, d = c1
    json.dump(g["lm"], open(d / "mlm_score.json", "w", encoding="utf-8"), ensure_ascii=False)
    json.dump(g["hyps_cer"], open(d / "hyps_cer.json", "w", encoding="utf-8"), ensure_ascii=False)
    feats = ["hyps_token_ids", "mlm_pll_score", "hyps_am_score", "hyps_cer"]
    fpaths = [str(d / f) for f in ("hyps_text.json", "mlm_score.json", "hyps_score.json", "hyps_cer.json")]

    def run(out, extra):
        return cli.rescorebert_train(cli.ArgParser().parse(["--config", _cfg(d, "MD_MWER_train.yaml", {
            "task": "training", "method": "MD_MWER", "seed": 10, "md_loss_weight": 0.0001, "lr": 1e-5, "epoch": 2,
            "device": "cuda:0", "random_init_seed": 1234, "train_feature": feats, "train_feature_path": fpaths,
            "dev_feature": feats, "dev_feature_path": fpaths, "output_path": str(out), "batch_size": 3,
            "max_utt": 99999999, "n_best": 10, "dataloader": {"shuffle": False, "num_worker": 5},
            "model": {"bert": "bert-base-chinese", "vocab": str(d / "vocab.txt")},
            "resume": extra})]))
    out = d / "train_out"
    res = run(out, {"start_from": None, "checkpoint_path": None})
    assert len(res["train_loss"]) == 2 and len(res["dev_loss"]) == 2
    assert all(np.isfinite(res["train_loss"])) and all(np.isfinite(res["dev_loss"]))
    assert [os.path.basename(p) for p in res["checkpoints"]] == ["checkpoint_1.pth", "checkpoint_2.pth"]
    rec = json.load(open(out / "loss.json", encoding="utf-8"))
    assert rec == {"train": res["train_loss"], "dev": res["dev_loss"]}
    sd = torch.load(res["checkpoints"][-1], map_location="cpu", weights_only=True)
    assert "linear.weight" in sd and "bert.pooler.dense.weight" in sd
    # resume (RescoreBert/main.py:185-200): epoch 2 from checkpoint_1.pth and loss.json
    out2 = d / "train_out_resume"
    out2.mkdir()
    json.dump({"train": res["train_loss"][:1], "dev": res["dev_loss"][:1]}, open(out2 / "loss.json", "w"))
    res2 = run(out2, {"start_from": 2, "checkpoint_path": res["checkpoints"][0]})
    assert res2["train_loss"] == res["train_loss"] and res2["dev_loss"] == res["dev_loss"]
    sd2 = torch.load(res2["checkpoints"][-1], map_location="cpu", weights_only=True)
    assert all(torch.equal(sd[k], sd2[k]) for k in sd)
    files = cli.rescorebert(cli.ArgParser().parse(["--config", _cfg(d, "MD_score.yaml", {
        "device": "cuda:0", "checkpoint_path": res["checkpoints"][-1], "n_best": 10,
        "model": {"bert": "bert-base-chinese", "vocab": str(d / "vocab.txt")},
        "dev_feature": ["hyps_token_ids"], "dev_feature_path": [str(d / "hyps_text.json")],
        "dev_output_format": str(d / "hyps_score.json"), "output_path": str(out)})]))
    lm = json.load(open(files["dev"], encoding="utf-8"))
    assert list(lm) == g["utt_ids"] and all(np.isfinite(v) for u in lm.values() for v in u.values())


def test_cli_mlm_finetune_then_pll(c1):
    """mlm_finetune with the reference's train.yaml layout (do_job rows JSON as
    train_data_path / dev_data_path, epoch, dataloader.batch_size / shuffle), then the
    checkpoint scores with mlm_pll."""
    import torch
    from asr_rescoring_amd import cli
    from asr_rescoring_amd.frontend import NativeTokenizer
    from asr_rescoring_amd.train import do_job_rows
    g, d = c1
    tok = NativeTokenizer(str(d / "vocab.txt"))
    rows = []
    for u, t in g["ref_text"].items():             # MLM_PLL/preprocess.py:9-30 "for_training" rows
        ids, off, lab = do_job_rows([[101] + tok.encode(t) + [102]])
        for i in range(len(off) - 1):
            r = ids[off[i]:off[i + 1]].tolist()
            rows.append({"utt_id": u, "hyp_id": None, "input_ids": r, "attention_masks": [1] * len(r),
                         "mask_pos": i + 1, "labels": lab[off[i]:off[i + 1]].tolist()})
    json.dump(rows, open(d / "train_rows.json", "w"))
    out = d / "mlm_out"
    res = cli.mlm_finetune(cli.ArgParser().parse(["--config", _cfg(d, "train.yaml", {
        "task": "training", "seed": 10, "lr": 1e-5, "epoch": 2, "device": "cuda:0", "random_init_seed": 1234,
        "train_data_path": str(d / "train_rows.json"), "dev_data_path": str(d / "train_rows.json"),
        "output_path": str(out), "num_of_data": 99999999,
        "dataloader": {"shuffle": False, "batch_size": 32, "num_worker": 5},
        "model": {"bert": "bert-base-chinese", "vocab": str(d / "vocab.txt")}})]))
    assert len(res["train_loss"]) == 2 and all(np.isfinite(res["train_loss"] + res["dev_loss"]))
    assert json.load(open(out / "loss.json")) == {"train": res["train_loss"], "dev": res["dev_loss"]}
    sd = torch.load(res["checkpoints"][-1], map_location="cpu", weights_only=True)
    assert os.path.basename(res["checkpoints"][-1]) == "checkpoint_2.pth"
    assert torch.equal(sd["cls.predictions.decoder.weight"], sd["bert.embeddings.word_embeddings.weight"])
    assert cli.main(["mlm_pll", "--config", _cfg(d, "score_ft.yaml", {
        "task": "scoring", "device": "cuda:0", "checkpoint_path": res["checkpoints"][-1],
        "train_hyps_text_path": str(d / "hyps_text.json"), "output_path": str(out) + "/",
        "model": {"bert": "bert-base-chinese", "vocab": str(d / "vocab.txt")}})]) == 0
    lm = json.load(open(str(out) + "/train_lm.json", encoding="utf-8"))
    assert list(lm) == g["utt_ids"] and all(np.isfinite(v) and v < 0 for u in lm.values() for v in u.values())


def test_cli_mlm_pll_two_ranks(c1, tmp_path):
    """``cli mlm_pll`` launched as 2 ranks (torchrun-style env, both on this box's GPU, gloo
    exchange since one GPU cannot host two RCCL ranks): utterance shards + one all-gather give
    the single-process scores (the C4 path of SURVEY §8e at toy scale)."""
    import socket
    import subprocess
    import sys
    from conftest import REPO
    g, d = c1
    outs = {}
    for world in (1, 2):
        out = tmp_path / f"w{world}"
        out.mkdir()
        cfg = _cfg(d, f"score_w{world}.yaml", {
            "task": "scoring", "device": "cuda:0", "random_init_seed": 1234,
            "train_hyps_text_path": str(d / "hyps_text.json"), "output_path": str(out) + "/",
            "model": {"bert": "bert-base-chinese", "vocab": str(d / "vocab.txt")}})
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        code = ("import sys; sys.path.insert(0, %r); import __graft_entry__ as g; g._import_pkg(); "
                "from asr_rescoring_amd import cli; sys.exit(cli.main(['mlm_pll', '--config', %r]))" % (REPO, cfg))
        procs = []
        for r in range(world):
            env = dict(os.environ, WORLD_SIZE=str(world), RANK=str(r), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=str(port), RS_DIST_BACKEND="gloo")
            procs.append(subprocess.Popen([sys.executable, "-c", code], env=env))
        for p in procs:
            assert p.wait(timeout=300) == 0
        outs[world] = json.load(open(out / "train_lm.json", encoding="utf-8"))
    assert list(outs[1]) == list(outs[2]) == g["utt_ids"]
    a = np.array([v for u in outs[1].values() for v in u.values()])
    b = np.array([v for u in outs[2].values() for v in u.values()])
    # the scores of a hypothesis do not depend on which rank / launch chunk computed them
    assert np.array_equal(a, b), np.abs(a - b).max()
