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


class _Replicas:
    """A strategy stand-in reporting W replicas (no process group: the selection logic only)."""

    def __init__(self, world):
        self.num_replicas_in_sync = world


def _trainer(name, hidden, world, **kw):
    import warnings

    from customknowledgegraphembedding_amd.model import TFKGEModel
    from customknowledgegraphembedding_amd.optim import Adam
    from customknowledgegraphembedding_amd.supervisor import Trainer
    from tests.shard_oracle_backend import OracleShardKernels

    m = TFKGEModel(name, 11, 2, hidden, 9.0, double_entity_embedding=name in ("InterHT", "RotatE"),
                   triple_relation_embedding=name == "InterHT", device="cpu", seed=0)
    with warnings.catch_warnings(record=True) as got:
        warnings.simplefilter("always")
        tr = Trainer(_Replicas(world), None, m, Adam(m.parameters(), lr=1e-3), Sum(),
                     shard_kernels=OracleShardKernels(), **kw)
    return tr, [str(w.message) for w in got]


def test_trainer_multi_replica_selection():
    """Across replicas the fused step row-shards the table only where the shard kernels run (per-half width
    <= 1024, not pRotatE); otherwise the dense all-reduce path runs, with a warning naming its bytes."""
    from customknowledgegraphembedding_amd.distributed import SHARD_MAX_D

    tr, warns = _trainer("InterHT", SHARD_MAX_D, 2)
    assert tr.fused and tr.sharded is not None and not warns
    tr, warns = _trainer("InterHT", SHARD_MAX_D + 1, 2)
    assert not tr.fused and tr.sharded is None
    assert len(warns) == 1 and "dense-gradient" in warns[0] and "MB" in warns[0] and "1025" in warns[0]
    tr, warns = _trainer("pRotatE", 8, 2)
    assert tr.sharded is None and len(warns) == 1 and "dense-gradient" in warns[0]
    tr, warns = _trainer("InterHT", SHARD_MAX_D + 1, 1)  # one replica: kge_train_step handles any width
    assert tr.fused and tr.sharded is None and not warns


def test_thread_comm_collectives_cpu():
    """ThreadComm's all-gather / all-to-all / all-reduce / broadcast between 3 threads equal the
    torch.distributed definitions (the simulated ranks of the single-GPU sharded runs)."""
    from customknowledgegraphembedding_amd.distributed import ThreadComm, run_threads

    W = 3
    comm = ThreadComm(W)

    def rank(r):
        c = comm.view(r)
        g = torch.empty(W, 2)
        c.all_gather_into(g, torch.tensor([r, 10.0 * r]))
        # rank r sends (r + 1) * d + 1 values to rank d, values 100 r + d
        ins = [(r + 1) * d + 1 for d in range(W)]
        inp = torch.cat([torch.full((n,), 100.0 * r + d) for d, n in enumerate(ins)])
        outs = [(s + 1) * r + 1 for s in range(W)]
        out = torch.empty(sum(outs))
        c.all_to_all(out, inp, outs, ins)
        s = c.all_reduce_sum_(torch.tensor([float(r + 1)]))
        b = c.broadcast_(torch.tensor([float(r)]), 2)
        return g, out, outs, s, b

    res = run_threads([lambda r=r: rank(r) for r in range(W)])
    for r, (g, out, outs, s, b) in enumerate(res):
        assert torch.equal(g, torch.tensor([[0.0, 0.0], [1.0, 10.0], [2.0, 20.0]]))
        want = torch.cat([torch.full((n,), 100.0 * src + r) for src, n in enumerate(outs)])
        assert torch.equal(out, want)
        assert float(s) == 6.0 and float(b) == 2.0


def test_from_model_with_thread_comm_copies_the_relation_table():
    """W simulated ranks of one process must not share one relation tensor (each applies the relation
    Adam update in place); the entity shards stay views of disjoint rows of the model's table."""
    from customknowledgegraphembedding_amd.distributed import ShardedKGE, ThreadComm
    from customknowledgegraphembedding_amd.model import TFKGEModel

    m = TFKGEModel("DistMult", 10, 3, 4, 9.0, device="cpu", seed=0)
    comm = ThreadComm(2)
    a = ShardedKGE.from_model(m, world=2, rank=0, comm=comm)
    b = ShardedKGE.from_model(m, world=2, rank=1, comm=comm)
    assert a.relation_embedding.data_ptr() != b.relation_embedding.data_ptr()
    assert a.relation_embedding.data_ptr() != m.relation_embedding.data_ptr()
    assert torch.equal(a.relation_embedding, m.relation_embedding.detach())
    assert a.shard.data_ptr() == m.entity_embedding.data_ptr()  # rows [0, 5): a view
