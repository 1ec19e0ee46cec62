"""train.py — the box-side driver with train_concap_struc.py's command line — on the GPU:

* parity: two optimizer steps on the recorded bs=2 batch of golden_bs2_hard (dropout off, the fixture's
  gumbel noise and LPM negatives, weights loaded through --file_state_dict) reproduce the reference
  model's losses within 1e-3 on BOTH steps (the first optimizer step runs at lr = 0, as the reference's
  LambdaLR does, so step 2 sees the same weights); the epoch's .bin / .tar land in the reference layout;
* loop: the native loader on raw product rows (char tokenizer, synthetic regions) through train + eval,
  finite losses, checkpoint written.
Each run is one subprocess (a fresh driver process, as on the command line)."""
import json
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest
import torch

from golden_util import CFG_PATH, HERE, REPO, load_case, case_config

pytestmark = pytest.mark.gpu


def _run(args, tmp_path, timeout=400):
    r = subprocess.run([sys.executable, os.path.join(REPO, "train.py")] + args, cwd=str(tmp_path),
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    return r


def _outdir(tmp_path):
    out = tmp_path / "out"
    out.mkdir()
    shutil.copy(CFG_PATH, out / "bert_base_6layer_6conect.json")
    return out


def test_train_py_parity_two_steps_match_golden(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k3m_amd.weights import param_values
    g = load_case("bs2_hard")
    out = _outdir(tmp_path)
    vals = param_values(case_config(g), int(g["weight_seed"]))
    torch.save({k: torch.from_numpy(v) for k, v in vals.items()}, str(tmp_path / "w.bin"))
    log = tmp_path / "loss.jsonl"
    _run(["--data_dir", str(tmp_path), "--output_dir", str(out), "--file_name", "unused", "--do_train",
          "--with_coattention", "--train_batch_size", "2", "--num_train_epochs", "1", "--if_pre_sampling", "1",
          "--file_state_dict", str(tmp_path / "w.bin"), "--k3m_parity_case",
          os.path.join(HERE, "golden", "golden_bs2_hard.npz"), "--k3m_max_steps", "2", "--k3m_loss_log", str(log)],
         tmp_path)
    rows = [json.loads(l) for l in log.read_text().splitlines()]
    assert len(rows) == 2
    ref = g["losses"]   # mlm_t, img, mlm_pv, lpm, nsp, loss
    for r in rows:
        got = np.array([r["masked_lm_loss"], r["masked_img_loss"], r["masked_lm_loss_pv"], r["loss_lpm"],
                        r["next_sentence_loss"], r["loss"]])
        np.testing.assert_allclose(got, ref, rtol=1e-3, atol=1e-4)
    assert rows[0]["lr"] >= 0.0
    ck_dir = out / "k3m_bert-base-uncased_12l_12h"
    assert (ck_dir / "hyperparamter.txt").exists()
    ck = torch.load(str(ck_dir / "K3M_struc_presample-1_epoch-0.tar"), map_location="cpu", weights_only=True)
    assert set(ck) == {"model_state_dict", "optimizer_state_dict", "scheduler_state_dict", "global_step"}
    assert ck["global_step"] == 2 and len(ck["model_state_dict"]) == 999
    sd = torch.load(str(ck_dir / "K3M_struc_presample-1_epoch-0.bin"), map_location="cpu", weights_only=True)
    # lr = 0 on the first step; the second step (lr = lr * lambda(1)) moved the weights
    assert not torch.equal(sd["struc_w1.weight"], torch.from_numpy(vals["struc_w1.weight"]))


def test_train_py_loader_loop_with_eval(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = _outdir(tmp_path)
    rows = []
    for i in range(6):
        pv = "#;#".join("p%d%d#:#v%d%d" % (i, j, j, i) for j in range(3 + i))
        rows.append("%d\titem title %d with words\thttp://img/%d.jpg\t%s\tcat" % (1000 + i, i, i, pv))
    for name in ("rows_train+valid.tsv", "rows_valid.tsv"):
        (tmp_path / name).write_text("\n".join(rows) + "\n", encoding="utf-8")
    log = tmp_path / "loss.jsonl"
    r = _run(["--data_dir", str(tmp_path), "--output_dir", str(out), "--file_name", "rows_{}.tsv", "--do_train",
              "--do_eval", "--with_coattention", "--train_batch_size", "3", "--eval_batch_size", "3",
              "--num_train_epochs", "1", "--k3m_char_tokenizer", "--k3m_synthetic_regions", "3",
              "--k3m_loss_log", str(log)], tmp_path)
    steps = [json.loads(l) for l in log.read_text().splitlines()]
    assert len(steps) == 2 and all(np.isfinite(s["loss"]) for s in steps)
    assert "[Eval] [Epoch-0] loss:" in r.stderr
    assert (out / "k3m_bert-base-uncased_12l_12h" / "K3M_struc_presample-1_epoch-0.bin").exists()
