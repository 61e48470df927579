"""End-to-end drop-in of tensorflow_codes/run.py on the GPU: sampler batches of the reference's countries_S1
triples -> TFRecord files (compress_data writer) -> run.main with the reference's flags (TFRecord reader,
TFKGEModel, Keras Adam + lrfn schedule, Trainer.training)."""
import os

import numpy as np
import pytest
import torch

from customknowledgegraphembedding_amd import run as R
from customknowledgegraphembedding_amd.sampler import TrainDataset
from customknowledgegraphembedding_amd.tfrecord import write_file_tfrecords

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_run_main_trains_from_tfrecords(tmp_path, capsys):
    z = np.load(os.path.join(GOLD, "countries_S1_train_ids.npz"))
    triples, E, Rn = z["triples"], int(z["nentity"]), int(z["nrelation"])
    B, N = 16, 4
    batches = []
    for mode in ("head-batch", "tail-batch"):
        ds = TrainDataset(triples, E, Rn, N, mode, seed=1)
        it = ds.batches(B, rng=np.random.RandomState(2))
        for _ in range(3):
            pos, neg, w, m = next(it)
            batches.append((pos.numpy(), neg.numpy(), w.numpy(), np.full(B, 0 if mode == "head-batch" else 1)))
    out = tmp_path / "countries"
    out.mkdir()
    paths = write_file_tfrecords(batches, str(out), B, split_number=2)
    model = R.main(["-ip", *paths, "-bz", str(B), "-sf", "TransE", "--nentity", str(E), "--nrelation", str(Rn),
                    "--hidden_dim", "50", "--gamma", "12", "--epochs", "2", "--steps_per_epoch", "3",
                    "--steps_per_tpu_call", "1"])
    text = capsys.readouterr().out
    assert "EPOCH 2/2" in text and "DONE" in text
    losses = [float(l.split("loss:")[1]) for l in text.splitlines() if "loss:" in l]
    assert len(losses) == 6 and all(np.isfinite(losses))
    assert torch.isfinite(model.entity_embedding).all()
