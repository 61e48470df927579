"""Training entry point with the reference's flags: tensorflow_codes/run.py on PyTorch-ROCm + libkge_hip.so.

    python -m customknowledgegraphembedding_amd.run -ip data.tfrec -bz 512 -sf InterHT --nentity 40943 \
        --nrelation 11 --hidden_dim 1000 --gamma 24 -de -tr --epochs 1 --steps_per_epoch 1000

Mirrors run.py:20-37 (args_parser), run.py:86-127 (run: TFRecord batches -> parse -> reshape -> repeat,
TFKGEModel, Keras Adam with the lrfn schedule, Sum metric, Trainer.training with steps_per_tpu_call=99) and
run.py:8-17 (check_device). One process per GPU; under torchrun the RCCL process group is joined and the
Trainer sums gradients over replicas like tf.distribute.
"""
from __future__ import annotations

import argparse
import os

import torch


def args_parser(argv=None):
    """run.py:20-37."""
    parser = argparse.ArgumentParser(description="Training ...")
    parser.add_argument("-ip", "--input_path", required=True, type=str, nargs="+")
    parser.add_argument("-bz", "--batch_size", required=True, type=int)
    parser.add_argument("-sf", "--score_function", required=True, type=str)
    parser.add_argument("--nentity", required=True, type=int)
    parser.add_argument("--nrelation", required=True, type=int)
    parser.add_argument("--hidden_dim", required=True, type=int)
    parser.add_argument("--gamma", required=True, type=float)
    parser.add_argument("--epochs", required=False, type=int, default=1)
    parser.add_argument("--steps_per_epoch", required=False, type=int, default=1000)
    parser.add_argument("-de", "--double_entity_embedding", action="store_true")
    parser.add_argument("-dr", "--double_relation_embedding", action="store_true")
    parser.add_argument("-tr", "--triple_relation_embedding", action="store_true")
    parser.add_argument("--steps_per_tpu_call", type=int, default=99,
                        help="step accounting of supervisor.py:41-42 (run.py:125 passes 99)")
    parser.add_argument("--seed", type=int, default=0, help="table initialisation seed (TF's RNG is not reproducible)")
    return parser.parse_args(argv)


def run(strategy, args):
    """run.py:86-127."""
    from .model import TFKGEModel
    from .optim import Adam, LRSchedule
    from .supervisor import Sum, Trainer
    from .tfrecord import load_batches

    dev = torch.device("cuda", torch.cuda.current_device())
    dataset = load_batches(args.input_path, args.batch_size, repeat=True, prefetch=2, pin_memory=True)
    with strategy.scope():
        kge_model = TFKGEModel(args.score_function, args.nentity, args.nrelation, args.hidden_dim, args.gamma,
                               double_entity_embedding=args.double_entity_embedding,
                               double_relation_embedding=args.double_relation_embedding,
                               triple_relation_embedding=args.triple_relation_embedding, device=dev, seed=args.seed)
        optimizer = Adam([p for p in kge_model.parameters() if p.requires_grad],
                         lr=LRSchedule(args.steps_per_epoch, strategy.num_replicas_in_sync))
        training_loss = Sum("training_loss")
        trainer = Trainer(strategy=strategy, dataloader=dataset, model=kge_model, optimizer=optimizer,
                          metrics=training_loss)
        trainer.training(steps_per_tpu_call=args.steps_per_tpu_call, epochs=args.epochs,
                         steps_per_epoch=args.steps_per_epoch)
    return kge_model


def main(argv=None):
    args = args_parser(argv)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as dist

        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from .supervisor import check_device

    strategy = check_device()
    model = run(strategy, args)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    return model


if __name__ == "__main__":
    main()
