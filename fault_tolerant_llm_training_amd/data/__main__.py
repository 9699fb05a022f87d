"""Dataset smoke test (reference ``dataset.py:104-166``).

    python -m fault_tolerant_llm_training_amd.data --dataset train.parquet \
        [--tokenizer-name-or-path byte] [--sequence-length 4096] [--batch-size 32]

Builds the map-style ParquetDataset + CollatorForCLM and the packing
IterableParquetDataset, prints a decoded sample, the batch shapes and the share
of label tokens ignored by the loss (-100), like the reference's ``__main__``.
"""
from __future__ import annotations

import argparse

from .loader import IterableSource, MapSource, TrainLoader
from .parquet import CollatorForCLM, IterableParquetDataset, ParquetDataset
from .tokenizer import encode, load_tokenizer, pad_token_id


def _report(name, inputs, labels):
    ignored = int((labels == -100).sum())
    total = labels.numel()
    print(f"[{name}] Input shape: {tuple(inputs.shape)}")
    print(f"[{name}] Labels shape: {tuple(labels.shape)}")
    print(f"[{name}] Ignored tokens in loss: {ignored} out of {total} ({ignored / total * 100:.2f}%)")


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--dataset", default="/capstor/store/cscs/ethz/large-sc/datasets/train_data.parquet")
    ap.add_argument("--tokenizer-name-or-path", default="unsloth/Mistral-Nemo-Base-2407-bnb-4bit")
    ap.add_argument("--sequence-length", type=int, default=4096)
    ap.add_argument("--batch-size", type=int, default=32)
    a = ap.parse_args(argv)
    tok = load_tokenizer(a.tokenizer_name_or_path)
    ds = ParquetDataset(a.dataset, tok, a.sequence_length, training_samples=a.batch_size)
    sample = ds[0]["input_ids"][:200]
    print(f"Decoded sample: {tok.decode(sample)}")
    col = CollatorForCLM(a.sequence_length, pad_token_id(tok))
    b = next(TrainLoader(MapSource(ds, col, a.batch_size, 0, 1), prefetch=0, pin=False))
    _report("ParquetDataset", b.inputs, b.labels)
    bos = getattr(tok, "bos_token_id", None)
    it = IterableParquetDataset(a.dataset, tok, a.sequence_length, bos_token_id=1 if bos is None else int(bos))
    b = next(TrainLoader(IterableSource(it, a.batch_size), prefetch=0, pin=False))
    _report("IterableParquetDataset", b.inputs, b.labels)
    print(f"IterableParquetDataset state after one batch: {it.state_dict()}")
    assert encode(tok, "x")  # tokenizer callable through the shared encode() path
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
