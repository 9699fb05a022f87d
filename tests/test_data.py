"""Datasets, collator and the prefetching loader (reference dataset.py:10-101)."""
import os

import pytest
import torch

from fault_tolerant_llm_training_amd.data.loader import IterableSource, MapSource, SyntheticSource, TrainLoader
from fault_tolerant_llm_training_amd.data.parquet import CollatorForCLM, IterableParquetDataset, ParquetDataset
from fault_tolerant_llm_training_amd.data.synthetic import SyntheticTokens
from fault_tolerant_llm_training_amd.data.tokenizer import ByteTokenizer, encode

from helpers import make_parquet


@pytest.fixture
def pq_file(tmp_path):
    p = str(tmp_path / "d.parquet")
    texts = make_parquet(p, n_docs=25)
    return p, texts


def hf_tokenizer(tmp_path):
    from tokenizers import Tokenizer, models, pre_tokenizers
    from transformers import AutoTokenizer, PreTrainedTokenizerFast

    vocab = {"[PAD]": 0, "<s>": 1, "[UNK]": 2}
    for w in ["alpha", "beta", "gamma", "delta", "eps", "zeta", "eta", "theta", "iota", "kappa"]:
        vocab[w] = len(vocab)
    t = Tokenizer(models.WordLevel(vocab, unk_token="[UNK]"))
    t.pre_tokenizer = pre_tokenizers.Whitespace()
    from tokenizers.processors import TemplateProcessing

    t.post_processor = TemplateProcessing(single="<s> $A", special_tokens=[("<s>", 1)])  # BOS like Mistral
    f = PreTrainedTokenizerFast(tokenizer_object=t, pad_token="[PAD]", bos_token="<s>", unk_token="[UNK]")
    d = str(tmp_path / "tok")
    f.save_pretrained(d)
    return AutoTokenizer.from_pretrained(d)


def test_collator_shift_and_mask():
    c = CollatorForCLM(sequence_length=4, pad_token_id=0)
    x, y = c([{"input_ids": [1, 5, 6, 0, 0]}, {"input_ids": [1, 7, 8, 9, 10]}])
    assert x.tolist() == [[1, 5, 6, 0], [1, 7, 8, 9]]
    assert y.tolist() == [[5, 6, -100, -100], [7, 8, 9, 10]]
    with pytest.raises(AssertionError):
        c([{"input_ids": [1, 2, 3]}])


@pytest.mark.parametrize("tok_kind", ["byte", "hf"])
def test_parquet_dataset(pq_file, tmp_path, tok_kind):
    path, texts = pq_file
    tok = ByteTokenizer() if tok_kind == "byte" else hf_tokenizer(tmp_path)
    ds = ParquetDataset(path, tok, sequence_length=16, training_samples=100)
    assert len(ds) == 100
    item = ds[30]  # wraps: row 30 % 25
    assert item["input_ids"] == encode(tok, texts[5], max_length=17, padding="max_length", truncation=True)
    assert len(item["input_ids"]) == 17


def _reference_packing(texts, tok, S, bos, n):
    """Re-statement of reference dataset.py:74-101 (plus the documented progress fix)."""
    out, idx = [], 0
    for _ in range(n):
        buf, docs = [], 0
        while len(buf) < S + 1:
            buf.extend(encode(tok, texts[idx % len(texts)], padding=False, truncation=True, max_length=S + 1))
            idx += 1
            docs += 1
        if docs > 1:  # progress fix for single over-long documents (see IterableParquetDataset)
            idx -= 1
        buf = buf[: S + 1]
        x, y = torch.tensor(buf[:-1]), torch.tensor(buf[1:])
        y[x == bos] = -100
        y[y == bos] = -100
        out.append((x, y))
    return out


@pytest.mark.parametrize("tok_kind", ["byte", "hf"])
def test_iterable_matches_reference_packing(pq_file, tmp_path, tok_kind):
    path, texts = pq_file
    tok = ByteTokenizer() if tok_kind == "byte" else hf_tokenizer(tmp_path)
    S = 24 if tok_kind == "byte" else 64
    ds = IterableParquetDataset(path, tok, S, bos_token_id=1)
    it = iter(ds)
    got = [next(it) for _ in range(12)]
    ref = _reference_packing(texts, tok, S, 1, 12)
    for (x, y), (rx, ry) in zip(got, ref):
        assert torch.equal(x, rx) and torch.equal(y, ry)
    assert (torch.stack([y for _, y in got]) == -100).any()  # BOS masking happened
    assert len({tuple(x.tolist()) for x, _ in got}) == len(got)  # always makes progress


def test_iterable_state_roundtrip_mid_shard(pq_file):
    path, _ = pq_file
    tok = ByteTokenizer()
    a = IterableParquetDataset(path, tok, 40)
    it = iter(a)
    for _ in range(7):
        next(it)
    sd = a.state_dict()
    tail = [next(it) for _ in range(5)]
    b = IterableParquetDataset(path, tok, 40)
    b.load_state_dict(sd)
    itb = iter(b)
    for (x, y), (x2, y2) in zip(tail, [next(itb) for _ in range(5)]):
        assert torch.equal(x, x2) and torch.equal(y, y2)


def test_iterable_sharding_disjoint_docs(pq_file):
    path, _ = pq_file
    tok = ByteTokenizer()
    r0 = IterableParquetDataset(path, tok, 16, rank=0, world_size=2)
    r1 = IterableParquetDataset(path, tok, 16, rank=1, world_size=2)
    assert [r0._row(i) for i in range(4)] == [0, 2, 4, 6]
    assert [r1._row(i) for i in range(4)] == [1, 3, 5, 7]
    with pytest.raises(ValueError):
        r1.load_state_dict({"current_index": 3, "world_size": 4})


@pytest.mark.parametrize("prefetch", [0, 2])
def test_loader_map_resume_is_exact(pq_file, prefetch):
    path, _ = pq_file
    tok = ByteTokenizer()
    ds = ParquetDataset(path, tok, 16, 10_000)
    col = CollatorForCLM(16, tok.pad_token_id)
    full = TrainLoader(MapSource(ds, col, 2, 0, 1), prefetch=prefetch, pin=False)
    batches = [next(full) for _ in range(9)]
    state = None
    l1 = TrainLoader(MapSource(ds, col, 2, 0, 1), prefetch=prefetch, pin=False)
    for _ in range(4):
        next(l1)
    state = l1.state_dict()
    l1.close()
    full.close()
    assert state == {"kind": "parquet", "next_step": 4}
    l2 = TrainLoader(MapSource(ds, col, 2, 0, 1), state=state, prefetch=prefetch, pin=False)
    for b_ref in batches[4:]:
        b = next(l2)
        assert b.step == b_ref.step and torch.equal(b.inputs, b_ref.inputs) and torch.equal(b.labels, b_ref.labels)
    l2.close()


def test_loader_iterable_state_is_last_consumed(pq_file):
    path, _ = pq_file
    tok = ByteTokenizer()

    def make():
        return IterableSource(IterableParquetDataset(path, tok, 20), 2)

    l1 = TrainLoader(make(), prefetch=3, pin=False)
    ref = [next(l1) for _ in range(8)]
    l1.close()
    l2 = TrainLoader(make(), prefetch=3, pin=False)
    for _ in range(3):
        next(l2)
    import time

    time.sleep(0.2)  # let the producer run ahead
    st = l2.state_dict()
    l2.close()
    assert st["next_step"] == 3
    l3 = TrainLoader(make(), state=st, prefetch=3, pin=False)
    for b_ref in ref[3:]:
        b = next(l3)
        assert b.step == b_ref.step and torch.equal(b.inputs, b_ref.inputs)
    l3.close()


def test_synthetic_sharding_and_counts():
    ds0 = SyntheticTokens(100, 8, seed=1, rank=0, world_size=2, pin=False)
    ds1 = SyntheticTokens(100, 8, seed=1, rank=1, world_size=2, pin=False)
    single = SyntheticTokens(100, 8, seed=1, pin=False)
    x0, _ = ds0.batch(3, 2)
    x1, _ = ds1.batch(3, 2)
    xs, _ = single.batch(3, 4)  # global batch of step 3 at world 1 with B*W samples
    assert torch.equal(torch.cat([x0, x1]), xs)
    b = next(TrainLoader(SyntheticSource(ds0, 2), prefetch=0, pin=False))
    assert b.num_items == 16


def test_loader_producer_error_surfaces(tmp_path):
    class Bad(SyntheticSource):
        def produce(self, step):
            raise RuntimeError("boom")

    l = TrainLoader(Bad(SyntheticTokens(10, 4, pin=False), 1), prefetch=2, pin=False)
    with pytest.raises(RuntimeError, match="boom"):
        next(l)
    l.close()
