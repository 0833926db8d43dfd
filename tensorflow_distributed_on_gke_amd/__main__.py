"""Command line entry point.

    python -m tensorflow_distributed_on_gke_amd train [--config FILE] [--set key=value ...] [--nproc N]
    python -m tensorflow_distributed_on_gke_amd test  --weights PREFIX [--sentence TEXT ...]
    python -m tensorflow_distributed_on_gke_amd heartbeat --port 3479

`train` is the reference's `python -m distributed_training_transformer`
(reference: distributed_training_transformer/__main__.py:1-186): in a
Kubernetes pod (THIS_POD_NAME set) it discovers the StatefulSet peers, runs
the heartbeat barrier and launches one training process per local GPU
(`--nproc`, default: all visible GPUs); locally it launches `--nproc`
processes on 127.0.0.1, or runs in-process when started by
torch.distributed.run (RANK set) or with one process.
`test` is the reference's test.py + Tester (greedy translation).
"""
from __future__ import annotations

import argparse
import os
import sys


def _visible_gpus() -> int:
    import torch

    return torch.cuda.device_count()  # does not initialise HIP


def cmd_train(args) -> int:
    from tensorflow_distributed_on_gke_amd.config import load_settings

    settings = load_settings(args.config if os.path.exists(args.config) else None, args.set)
    in_child = "RANK" in os.environ
    if not in_child:
        from tensorflow_distributed_on_gke_amd.cluster import launch, rendezvous

        nproc = args.nproc if args.nproc > 0 else max(1, _visible_gpus())
        pod = os.environ.get("THIS_POD_NAME")
        if pod or nproc > 1:
            spec = rendezvous.bootstrap(settings.worker_count if pod else 1, namespace=args.namespace,
                                        heartbeat_port=args.heartbeat_port, master_port=args.master_port,
                                        verbose=True)
            argv = ["-m", "tensorflow_distributed_on_gke_amd", "train", "--config", args.config]
            for kv in args.set or []:
                argv += ["--set", kv]
            rc = launch.launch(argv, nproc, spec)
            if rc == 0 and settings.idle_after_train:
                from tensorflow_distributed_on_gke_amd.train.loop import idle_forever

                idle_forever()
            return rc
    from tensorflow_distributed_on_gke_amd.parallel import dist as tdist
    from tensorflow_distributed_on_gke_amd.train.loop import Trainer, idle_forever

    info = tdist.init_distributed(args.device)
    if info.chief:
        print(f"Number of devices: {info.world}", flush=True)
    trainer = Trainer(settings, info, log=lambda m: print(m, flush=True))
    trainer.fit()
    if trainer.ddp is not None:
        trainer.ddp.close()
    tdist.shutdown()
    if settings.idle_after_train and not in_child:
        idle_forever()
    return 0


def cmd_test(args) -> int:
    import torch

    from tensorflow_distributed_on_gke_amd.checkpoint import bundle
    from tensorflow_distributed_on_gke_amd.config import load_settings
    from tensorflow_distributed_on_gke_amd.infer.greedy import Tester
    from tensorflow_distributed_on_gke_amd.infer.tokenizer import ByteTokenizer
    from tensorflow_distributed_on_gke_amd.train.loop import build_model

    settings = load_settings(args.config if os.path.exists(args.config) else None, args.set)
    dev = args.device if args.device != "auto" else ("cuda:0" if torch.cuda.is_available() else "cpu")
    if settings.src_tokenizer and settings.tgt_tokenizer:
        # the WordPiece pair a text-data training run saved (data/text.py); like
        # the reference, the vocabulary sizes come from the tokenizers
        from types import SimpleNamespace

        from tensorflow_distributed_on_gke_amd.data.text import WordPieceTokenizer
        pt = WordPieceTokenizer.load(settings.src_tokenizer)
        en = WordPieceTokenizer.load(settings.tgt_tokenizer)
        settings.src_vocab, settings.tgt_vocab = pt.vocab_size, en.vocab_size
        tok = SimpleNamespace(pt=pt, en=en)
    else:
        tok = ByteTokenizer(min(settings.src_vocab, settings.tgt_vocab))
    model = build_model(settings, dev)
    if args.weights:
        bundle.load_weights(model.store, args.weights)
    tester = Tester(tok, model)
    text, tokens, attn = tester(list(args.sentence), max_length=args.max_length)
    for s, t in zip(args.sentence, text):
        print(f"{s!r} -> {t!r}")
    print("attention maps:", {k: tuple(v.shape) for k, v in attn.items()})
    return 0


def cmd_heartbeat(args) -> int:
    import time

    from tensorflow_distributed_on_gke_amd.cluster.heartbeat import start_heartbeat_server

    start_heartbeat_server(args.port)
    print(f"heartbeat server on :{args.port}", flush=True)
    while True:
        time.sleep(3600)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="tensorflow_distributed_on_gke_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    common = argparse.ArgumentParser(add_help=False)
    common.add_argument("--config", default="configuration/settings.yaml")
    common.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    common.add_argument("--device", default="auto")
    t = sub.add_parser("train", parents=[common])
    t.add_argument("--nproc", type=int, default=0, help="processes (GPUs) per node; 0 = all visible")
    t.add_argument("--namespace", default=os.environ.get("POD_NAMESPACE", "default"))
    t.add_argument("--heartbeat-port", type=int, default=3479)
    t.add_argument("--master-port", type=int, default=int(os.environ.get("MASTER_PORT", 3480)))
    e = sub.add_parser("test", parents=[common])
    e.add_argument("--weights", default=None, help="weights prefix or directory")
    e.add_argument("--sentence", action="append", default=None)
    e.add_argument("--max-length", type=int, default=20)
    h = sub.add_parser("heartbeat")
    h.add_argument("--port", type=int, default=3479)
    args = ap.parse_args(argv)
    if args.cmd == "test" and not args.sentence:
        args.sentence = ["muitas pessoas vieram à estação."]  # reference test.py:9
    return {"train": cmd_train, "test": cmd_test, "heartbeat": cmd_heartbeat}[args.cmd](args)


if __name__ == "__main__":
    sys.exit(main())
