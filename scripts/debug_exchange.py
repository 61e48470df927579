"""Stage-by-stage check of the row-sharded exchange kernels against the CPU restatement
(tests/shard_oracle_backend.py) on one GPU, W ranks as threads (debug aid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import customknowledgegraphembedding_amd as kge  # noqa: E402
from customknowledgegraphembedding_amd.distributed import HipShardKernels as HK, ShardedKGE, ThreadComm  # noqa: E402
from tests.shard_oracle_backend import OracleShardKernels as OK  # noqa: E402

name, E, R, d, W, K, Bh, N = "TransE", 997, 6, 40, 2, 2, 6, 37
mode = int(sys.argv[1]) if len(sys.argv) > 1 else 0
m = kge.TFKGEModel(name, E, R, d, 9.0, device="cuda", seed=3)
g = np.random.RandomState(1)
Bg = W * Bh
pos = torch.from_numpy(np.stack([g.randint(E, size=Bg), g.randint(R, size=Bg), g.randint(E, size=Bg)], 1)).cuda()
neg = torch.from_numpy(g.randint(E, size=(Bg, N))).cuda()
tables = (m.entity_embedding.detach(), m.relation_embedding.detach(), m._gamma_f, m._range_f, 0.0)
comm = ThreadComm(W)
ranks = [ShardedKGE(name, E, R, d, 9.0, device="cuda", world=W, rank=r, comm=comm, full_tables=tables) for r in range(W)]
plans = [HK.plan(sk, pos, neg, mode, K) for sk in ranks]  # identical but for each rank's bucket
plan = plans[0]
tot, qtot = plan.summary()
print("tot", tot.tolist(), "qtot", qtot.tolist())
Rk, hpc = Bg // K, W // K
for k in range(K):
    per = [int(qtot[k, :, o].sum()) for o in range(W)]
    parts, qidx_d = [], None
    for sk in ranks:
        snd = torch.empty((W, per[sk.rank], d), device="cuda")
        qidx = torch.empty((plan.ncol, Rk), dtype=torch.int64, device="cuda")
        HK.gather_queries(sk, plans[sk.rank], pos, k, snd, qidx)
        snd_o = torch.zeros((W, per[sk.rank], d))
        qidx_o = torch.zeros((plan.ncol, Rk), dtype=torch.int64)
        skc = ShardedKGE(name, E, R, d, 9.0, device="cpu", world=W, rank=sk.rank,
                         full_tables=tuple(x.cpu() if torch.is_tensor(x) else x for x in tables))
        plan_c = OK.plan(skc, pos.cpu(), neg.cpu(), mode, K)
        OK.gather_queries(skc, plan_c, pos.cpu(), k, snd_o, qidx_o)
        print("chunk", k, "rank", sk.rank, "send equal", torch.equal(snd.cpu(), snd_o), "qidx equal",
              torch.equal(qidx.cpu(), qidx_o), qidx.cpu().tolist(), qidx_o.tolist())
        parts.append(snd[0])
        qidx_d = qidx
    block = torch.cat(parts)
    for sk in ranks:
        n_send = int(sum(tot[h, sk.rank] for h in range(k * hpc, (k + 1) * hpc)))
        send = torch.full((n_send,), -7.0, device="cuda")
        HK.score_compact(sk, block, qidx_d[0], pos, neg, plans[sk.rank], k * Rk, Rk, send)
        skc = ShardedKGE(name, E, R, d, 9.0, device="cpu", world=W, rank=sk.rank,
                         full_tables=tuple(x.cpu() if torch.is_tensor(x) else x for x in tables))
        plan_c = OK.plan(skc, pos.cpu(), neg.cpu(), mode, K)
        send_o = torch.full((n_send,), -7.0, dtype=torch.float64)
        OK.score_compact(skc, block.cpu(), qidx_d[0].cpu(), pos.cpu(), neg.cpu(), plan_c, k * Rk, Rk, send_o)
        diff = (send.cpu().double() - send_o).abs()
        print("chunk", k, "rank", sk.rank, "send", n_send, "max diff", float(diff.max()) if n_send else 0,
              "bad idx", (diff > 1e-4).nonzero().reshape(-1)[:10].tolist())
