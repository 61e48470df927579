"""Training-step driver: mirror of tensorflow_codes/supervisor.py (Trainer) and run.py:8-17
(check_device) on PyTorch-ROCm.

`Trainer.train_step` is the caller of the hot path: the two model calls of supervisor.py:17-18 run
as one fused `TFKGEModel.step_forward` (2 HIP launches), the loss is supervisor.py:19-23, the
backward runs the HIP backward kernels, and the optimizer (customknowledgegraphembedding_amd.optim.Adam)
runs the HIP Adam kernel.

Multi-replica (torch.distributed, one process per GPU): the step is the same math as tf.distribute's
(supervisor.py:26-28): each replica's loss on its own batch, the replicas' gradients SUM-aggregated
by `apply_gradients`, `metrics` += loss * num_replicas_in_sync. With the fused optimizer the entity
table is ROW-SHARDED over the replicas for the step (distributed.ShardedKGE.train_step: owner-computes,
each rank updates its block of rows in place, collectives of O(batch) size instead of a dense
all-reduce of the whole table's gradient); the replicas' batches are all-gathered (ids and weights).
Otherwise the dense table gradients are summed with all-reduce before the optimizer step.
"""
from __future__ import annotations

import contextlib
import time

import torch


class Strategy:
    """The part of a tf.distribute strategy the reference uses (run.py:8-17, supervisor.py:28-30)."""

    def __init__(self):
        import torch.distributed as dist

        self._dist = dist if (dist.is_available() and dist.is_initialized()) else None
        self.num_replicas_in_sync = self._dist.get_world_size() if self._dist else 1

    def scope(self):
        return contextlib.nullcontext()

    def run(self, fn, args=()):
        return fn(*args)

    def sum_over_replicas(self, t):
        """The SUM of a (small) tensor over the replicas."""
        if self._dist is None or self.num_replicas_in_sync == 1:
            return t
        t = t.clone()
        self._dist.all_reduce(t, op=self._dist.ReduceOp.SUM)
        return t

    def all_reduce_grads(self, params):
        if self._dist is None or self.num_replicas_in_sync == 1:
            return
        for p in params:
            if p.grad is not None:
                self._dist.all_reduce(p.grad, op=self._dist.ReduceOp.SUM)


def check_device() -> Strategy:
    """run.py:8-17: the strategy for the visible accelerators."""
    s = Strategy()
    print("Number of accelerators: ", s.num_replicas_in_sync)
    return s


class Sum:
    """tf.keras.metrics.Sum (run.py:114): accumulates on device, reads back on result()."""

    def __init__(self, name="training_loss"):
        self.name = name
        self._total = None

    def update_state(self, value):
        v = value.detach().to(torch.float32).reshape(())
        self._total = v.clone() if self._total is None else self._total + v

    def accumulator(self, device):
        """The running total as a 0-dim fp32 device tensor that a kernel adds into in place
        (kge_train_step's loss_sum)."""
        if self._total is None:
            self._total = torch.zeros((), dtype=torch.float32, device=device)
        return self._total

    def result(self):
        return torch.tensor(0.0) if self._total is None else self._total.detach().cpu()

    def reset_states(self):
        self._total = None


class Trainer:
    """supervisor.py:5-58."""

    def __init__(self, strategy, dataloader, model, optimizer, metrics, fused=None, shard_kernels=None):
        self.dataloader = dataloader
        self.model = model
        self.optimizer = optimizer
        self.metrics = metrics
        self.strategy = strategy
        replicas = strategy.num_replicas_in_sync
        if fused is None:
            # the fused optimizer never materialises gradients: it needs this package's Adam over
            # exactly the model's parameters in one group (and, across replicas, no pRotatE modulus)
            from .optim import Adam
            fused = (isinstance(optimizer, Adam)
                     and hasattr(model, "train_step_fused") and getattr(model, "supports_fused_step", False)
                     and len(optimizer.param_groups) == 1
                     and {id(p) for p in optimizer.param_groups[0]["params"] if p.requires_grad}
                     == {id(p) for p in model.parameters() if p.requires_grad}
                     and (replicas == 1 or model.model_name != "pRotatE"))
        # fused="split": the three-call form (kge_step_forward, kge_step_loss, kge_step_backward_adam),
        # bitwise equal to the autograd path; otherwise the single kge_train_step call
        self.one_call = fused != "split"
        self.fused = bool(fused)
        self.sharded = None
        if replicas > 1:
            from .distributed import SHARD_MAX_D, ShardedKGE, warn_dense_fallback
            if self.fused and fused == "split":
                raise ValueError("fused='split' is single-replica only")
            D = int(getattr(model, "_D", 0))
            if self.fused and D > SHARD_MAX_D:
                # the row-sharded kernels keep six accumulators per element in registers (D <= 1024
                # per half); the dense all-reduce path below has no such limit
                self.fused = False
                warn_dense_fallback(model, replicas, f"per-half width {D} > {SHARD_MAX_D}")
            elif self.fused:
                self.sharded = ShardedKGE.from_model(model, kernels=shard_kernels)
            else:
                warn_dense_fallback(model, replicas, "no fused step for this model / optimizer")

    def loss(self, positive_sample, negative_sample, subsampling_weight, mode):
        """supervisor.py:17-23 — both calls fused, then the weighted loss (one HIP launch each)."""
        from . import ops

        negative_score, positive_score = self.model.step_forward(positive_sample, negative_sample, mode[0])
        return ops.step_loss(negative_score, positive_score, subsampling_weight)  # kge_step_loss

    def train_step(self, data_iter):
        """supervisor.py:13-30."""

        def train_step_fn(positive_sample, negative_sample, subsampling_weight, mode):
            dev = self.model.entity_embedding.device
            positive_sample = positive_sample.to(dev, non_blocking=True)
            negative_sample = negative_sample.to(dev, non_blocking=True)
            subsampling_weight = subsampling_weight.to(dev, non_blocking=True)
            mode = mode.cpu() if torch.is_tensor(mode) else mode
            if self.sharded is not None:
                return self._sharded_step(positive_sample, negative_sample, subsampling_weight, mode)
            if self.fused:
                # forward + loss + deterministic backward with Adam fused into the entity pass
                acc = (self.metrics.accumulator(dev) if self.one_call and hasattr(self.metrics, "accumulator")
                       else None)  # single replica: the metric update happens inside the step's last kernel
                loss = self.model.train_step_fused(positive_sample, negative_sample, subsampling_weight, mode[0],
                                                   self.optimizer, one_call=self.one_call, loss_sum=acc)
                if acc is None:
                    self.metrics.update_state(loss * self.strategy.num_replicas_in_sync)
                return loss
            self.optimizer.zero_grad(set_to_none=True)
            loss = self.loss(positive_sample, negative_sample, subsampling_weight, mode)
            loss.backward()                                                    # :25
            self.strategy.all_reduce_grads(self.model.parameters())
            self.optimizer.step()                                              # :26
            # :28 under tf.distribute: every replica adds loss * num_replicas_in_sync to a Sum metric
            # whose read is the cross-replica SUM, so the metric is W * (sum of the replicas' losses),
            # as the row-sharded path records it
            self.metrics.update_state(self.strategy.sum_over_replicas(loss.detach())
                                      * self.strategy.num_replicas_in_sync)
            return loss.detach()  # the backward has run; the value is what the caller reads

        return self.strategy.run(train_step_fn, next(data_iter))

    def _sharded_step(self, pos, neg, w, mode):
        """supervisor.py:15-28 across the replicas with the entity table row-sharded: the replicas'
        batches are all-gathered (every replica must be in the same negative mode this step), then
        ShardedKGE.train_step (Keras/torch Adam from this optimizer's group, in place on the model)."""
        from . import ops
        from .optim import resolve_lr

        sk = self.sharded
        comm = sk.comm
        m0 = ops.mode_id(int(mode[0]) if torch.is_tensor(mode) or isinstance(mode, (list, tuple)) else mode)
        modes = comm.all_gather_cat(torch.tensor([m0], dtype=torch.int64, device=pos.device)).reshape(-1)
        if bool((modes != modes[0]).any()):
            raise ValueError(f"replicas are in different negative modes this step: {modes.tolist()}")
        pos_g = comm.all_gather_cat(pos.contiguous()).reshape(-1, 3)
        neg_g = comm.all_gather_cat(neg.contiguous())
        neg_g = neg_g.reshape(-1, neg_g.shape[-1])
        w_g = comm.all_gather_cat(w.reshape(-1).to(torch.float32).contiguous()).reshape(-1)
        ent, rel = self.model.entity_embedding, self.model.relation_embedding
        group = self.optimizer.param_groups[0]
        for prm in (ent, rel):
            st = self.optimizer.state[prm]
            if not st:
                st["step"] = 0
                st["exp_avg"] = torch.zeros_like(prm)
                st["exp_avg_sq"] = torch.zeros_like(prm)
        st_e, st_r = self.optimizer.state[ent], self.optimizer.state[rel]
        sk.adam = {"m_ent": st_e["exp_avg"][sk.lo:sk.hi], "v_ent": st_e["exp_avg_sq"][sk.lo:sk.hi],
                   "m_rel": st_r["exp_avg"], "v_rel": st_r["exp_avg_sq"],
                   "lr": resolve_lr(group["lr"], st_e["step"]), "b1": group["betas"][0], "b2": group["betas"][1],
                   "eps": group["eps"], "keras": group["semantics"] == "keras"}
        sk.step = st_e["step"]
        loss = sk.train_step(pos_g, neg_g, w_g, m0)
        st_e["step"] += 1
        st_r["step"] += 1
        # supervisor.py:28: every replica adds loss * num_replicas_in_sync to the (cross-replica SUM) metric
        # (ShardedKGE.loss_sum stays None on this path: the metric is updated here, not inside the step)
        self.metrics.update_state(sk.last_losses.sum() * self.strategy.num_replicas_in_sync)
        return loss

    def sync_model(self):
        """After sharded training: every rank's block of entity rows back into the model's table. The
        Adam moments are NOT re-broadcast: each rank advances only its own rows of the optimizer's
        exp_avg / exp_avg_sq (views of the shard), so a state_dict taken mid-training is current on the
        rank's own rows only."""
        if self.sharded is not None:
            self.sharded.sync_entity_table(self.model.entity_embedding.data)

    def training(self, steps_per_tpu_call, epochs, steps_per_epoch):
        """supervisor.py:32-58. Reproduces the reference loop, including its step accounting
        (`step += steps_per_tpu_call` per single train_step call, supervisor.py:41-42)."""
        step = 0
        epoch = 0
        epoch_start_time = time.time()
        iteration_data = iter(self.dataloader)
        while True:
            self.train_step(iteration_data)
            step += steps_per_tpu_call
            print("=", end="", flush=True)
            epoch_time = time.time() - epoch_start_time
            print("\nEPOCH {:d}/{:d}".format(epoch + 1, epochs))
            print("time: {:0.1f}s".format(epoch_time),
                  "loss: {:0.4f}".format(round(float(self.metrics.result()), 4)), flush=True)
            epoch = step // steps_per_epoch
            epoch_start_time = time.time()
            self.metrics.reset_states()
            if epoch >= epochs:
                break
        self.sync_model()
        print("DONE")
