"""CPU tests of the host-side training driver pieces (no GPU calls)."""
import torch

from customknowledgegraphembedding_amd.supervisor import Strategy, Sum, check_device
from oracle import kge_oracle as O


def test_strategy_single_process():
    s = check_device()
    assert s.num_replicas_in_sync == 1
    assert s.run(lambda a, b: a + b, (2, 3)) == 5


def test_sum_metric():
    m = Sum()
    m.update_state(torch.tensor(1.5))
    m.update_state(torch.tensor([2.0]))
    assert float(m.result()) == 3.5
    m.reset_states()
    assert float(m.result()) == 0.0


def test_lrfn_schedule_run_py():
    # run.py:69-84
    assert abs(O.lrfn(0) - 1e-5) < 1e-12
    assert abs(O.lrfn(5) - 5e-5) < 1e-12
    assert abs(O.lrfn(6) - ((5e-5 - 1e-5) * 0.8 + 1e-5)) < 1e-12
    assert abs(O.lrfn(0, num_replicas=8) - 1e-5) < 1e-12
    assert abs(O.lrfn(5, num_replicas=8) - 4e-4) < 1e-12


def test_lr_schedule_matches_reference_formula():
    """run.py:69-84 (lrfn) and :106-108 (LRSchedule: epoch = step // steps_per_epoch)."""
    from customknowledgegraphembedding_amd.optim import LRSchedule, lrfn, resolve_lr
    from oracle import kge_oracle as O

    for e in range(12):
        assert lrfn(e) == O.lrfn(e)
        assert lrfn(e, 8) == O.lrfn(e, 8)
    s = LRSchedule(steps_per_epoch=100)
    assert resolve_lr(s, 0) == lrfn(0) and resolve_lr(s, 250) == lrfn(2)
    assert resolve_lr(lambda: 0.5, 7) == 0.5 and resolve_lr(0.25, 3) == 0.25


def test_run_args_parser_matches_reference_flags():
    """tensorflow_codes/run.py:20-37 flags (short and long forms)."""
    from customknowledgegraphembedding_amd.run import args_parser

    a = args_parser(["-ip", "x.tfrec", "-bz", "512", "-sf", "InterHT", "--nentity", "40943", "--nrelation", "11",
                     "--hidden_dim", "1000", "--gamma", "24", "-de", "-tr"])
    assert (a.input_path, a.batch_size, a.score_function) == (["x.tfrec"], 512, "InterHT")
    assert a.double_entity_embedding and a.triple_relation_embedding and not a.double_relation_embedding
    assert (a.epochs, a.steps_per_epoch, a.steps_per_tpu_call) == (1, 1000, 99)
