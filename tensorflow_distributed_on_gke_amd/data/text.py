"""Real-text translation pairs: the reference's dataset pipeline on local files.

Reference (distributed_training_transformer/english_portugese_dataset.py:8-51):
TFDS `ted_hrlr_translate/pt_to_en`, tokenized by the `ted_hrlr_translate_pt_en_converter`
SavedModel (a BERT-style WordPiece tokenizer per language with the reserved
tokens [PAD] [UNK] [START] [END]), pipeline `cache -> shuffle(20000) ->
batch(GLOBAL_BATCH) -> map(tokenize -> .to_tensor()) -> prefetch`, auto-sharded
with `AutoShardPolicy.DATA`; the vocabulary sizes are probed from the
tokenizers at start-up (__main__.py:32-35).

Here (no TensorFlow, no network):

* `WordPieceTokenizer` -- the same tokenizer family, trained from the training
  corpus with the HF `tokenizers` library (BERT normalisation / pre-tokenisation,
  `##` continuation pieces, the same four reserved ids 0..3) or loaded from a
  saved JSON; it also has the Tester's tokenizer interface (infer/tokenizer.py).
  Vocabulary ids are not the reference converter's (its SavedModel is not
  loadable without TensorFlow): parity of the tokenisation itself is unpinned.
* `TextPairs` -- a TSV file of `source<TAB>target` lines, tokenised once
  (`cache`), a seeded buffered shuffle of 20000 pairs re-drawn every epoch
  (tf.data's reshuffle_each_iteration), global batches of local_batch x world
  pairs, each rank taking its contiguous slice (the DATA shard of the global
  batch), each global batch right-padded with PAD to its longest sequence
  (`.to_tensor()`). Pairs longer than max_len tokens are dropped (the
  reference would fail on them: positional tables of length 1000).
  `bucket` > 1 pads further, to the next multiple of `bucket` (source) and
  of `bucket` + the one shifted token (target), capped at max_len, so the
  batch shapes fall into few buckets and the HIP-graph step cache
  (train/step.py) replays a captured step for most batches.
"""
from __future__ import annotations

import os
import random
from typing import Iterable, Iterator, List, Optional, Sequence, Tuple, Union

import torch

PAD, UNK, START, END = 0, 1, 2, 3
RESERVED = ["[PAD]", "[UNK]", "[START]", "[END]"]


class WordPieceTokenizer:
    """BERT-style WordPiece with the reference converter's reserved tokens."""

    def __init__(self, tok):
        self._tok = tok
        for i, name in enumerate(RESERVED):
            if tok.token_to_id(name) != i:
                raise ValueError(f"tokenizer must map {name} to id {i}")

    # ------------------------------------------------------------ construction
    @classmethod
    def train(cls, texts: Iterable[str], vocab_size: int, lowercase: bool = True) -> "WordPieceTokenizer":
        from tokenizers import Tokenizer, decoders, models, normalizers, pre_tokenizers, trainers

        tok = Tokenizer(models.WordPiece(unk_token="[UNK]"))
        tok.normalizer = normalizers.BertNormalizer(lowercase=lowercase, strip_accents=False)
        tok.pre_tokenizer = pre_tokenizers.BertPreTokenizer()
        tok.decoder = decoders.WordPiece()
        trainer = trainers.WordPieceTrainer(vocab_size=vocab_size, special_tokens=RESERVED,
                                            show_progress=False)
        tok.train_from_iterator(texts, trainer)
        return cls(tok)

    @classmethod
    def load(cls, path: str) -> "WordPieceTokenizer":
        from tokenizers import Tokenizer

        return cls(Tokenizer.from_file(path))

    def save(self, path: str) -> None:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self._tok.save(path)

    # ------------------------------------------------------------ interface
    @property
    def vocab_size(self) -> int:
        return self._tok.get_vocab_size()

    def start_end(self):
        return START, END

    def encode(self, text: str, add_start_end: bool = True) -> List[int]:
        ids = self._tok.encode(text, add_special_tokens=False).ids
        return [START] + ids + [END] if add_start_end else ids

    def encode_batch(self, texts: Sequence[str]) -> List[List[int]]:
        return [[START] + e.ids + [END]
                for e in self._tok.encode_batch(list(texts), add_special_tokens=False)]

    def tokenize(self, texts: Union[str, Sequence[str]]) -> torch.Tensor:
        """Right-padded int64 [B, L] with [START] ... [END] (the Tester API)."""
        if isinstance(texts, str):
            texts = [texts]
        return pad_rows(self.encode_batch(texts))

    def lookup(self, ids: Sequence[int]) -> List[str]:
        return [self._tok.id_to_token(int(i)) or f"<{int(i)}>" for i in ids]

    def detokenize(self, ids: Sequence[int]) -> str:
        return self._tok.decode([int(i) for i in ids if int(i) > END], skip_special_tokens=True)


def pad_rows(rows: Sequence[Sequence[int]], length: Optional[int] = None) -> torch.Tensor:
    L = length if length is not None else max(len(r) for r in rows)
    out = torch.full((len(rows), L), PAD, dtype=torch.int64)
    for i, r in enumerate(rows):
        out[i, : len(r)] = torch.tensor(r, dtype=torch.int64)
    return out


def bucket_lengths(S: int, T: int, bucket: int, max_len: int) -> Tuple[int, int]:
    """Padded (source, target) lengths of a batch whose longest rows are S
    and T tokens: the source to a multiple of `bucket`, the target so that
    the teacher-forced decoder input (T - 1 tokens) is one; both capped at
    max_len (longer pairs were dropped, so the cap never cuts a row)."""
    if bucket <= 1:
        return S, T
    Sb = min(-(-S // bucket) * bucket, max(S, max_len))
    Tb = min(-(-(T - 1) // bucket) * bucket + 1, max(T, max_len))
    return Sb, Tb


def read_pairs(path: str) -> List[Tuple[str, str]]:
    """`source<TAB>target` lines (blank lines and lines without a tab skipped)."""
    pairs = []
    with open(path, encoding="utf-8") as f:
        for line in f:
            line = line.rstrip("\n")
            if "\t" not in line:
                continue
            s, t = line.split("\t", 1)
            if s.strip() and t.strip():
                pairs.append((s.strip(), t.strip()))
    return pairs


def build_tokenizers(train_path: str, src_vocab: int, tgt_vocab: int, cache_dir: Optional[str] = None,
                     src_path: Optional[str] = None, tgt_path: Optional[str] = None):
    """Load the two tokenizers, or train them on the training corpus (and save
    them under cache_dir). Their vocabulary sizes size the model, as the
    reference probes its converter's vocabularies (__main__.py:32-35)."""
    if src_path and tgt_path and os.path.exists(src_path) and os.path.exists(tgt_path):
        return WordPieceTokenizer.load(src_path), WordPieceTokenizer.load(tgt_path)
    pairs = read_pairs(train_path)
    src = WordPieceTokenizer.train((p[0] for p in pairs), src_vocab)
    tgt = WordPieceTokenizer.train((p[1] for p in pairs), tgt_vocab)
    if cache_dir:
        src.save(os.path.join(cache_dir, "tokenizer_src.json"))
        tgt.save(os.path.join(cache_dir, "tokenizer_tgt.json"))
    return src, tgt


def buffered_shuffle(n: int, buffer: int, seed: int) -> List[int]:
    """The order tf.data's shuffle(buffer) emits indices 0..n-1 in: fill a
    buffer, emit a random slot and refill it from the stream, drain at the end."""
    rng = random.Random(seed)
    buf = list(range(min(buffer, n)))
    nxt = len(buf)
    out = []
    while buf:
        j = rng.randrange(len(buf))
        out.append(buf[j])
        if nxt < n:
            buf[j] = nxt
            nxt += 1
        else:
            buf[j] = buf[-1]
            buf.pop()
    return out


class TextPairs:
    """Tokenised (source, target) pairs batched like the reference pipeline;
    the same next / seek / batch interface as SyntheticPairs."""

    def __init__(self, path: str, src_tok, tgt_tok, local_batch: int, rank: int = 0, world: int = 1,
                 seed: int = 0, shuffle_buffer: int = 20000, shuffle: bool = True,
                 max_len: int = 1000, pin: bool = False, bucket: int = 1):
        pairs = read_pairs(path)
        src_ids = src_tok.encode_batch([p[0] for p in pairs])
        tgt_ids = tgt_tok.encode_batch([p[1] for p in pairs])
        keep = [i for i in range(len(pairs)) if len(src_ids[i]) <= max_len and len(tgt_ids[i]) <= max_len]
        self.src = [src_ids[i] for i in keep]  # the tf.data `cache()`
        self.tgt = [tgt_ids[i] for i in keep]
        self.dropped = len(pairs) - len(keep)
        self.local_batch, self.rank, self.world = local_batch, rank, world
        self.global_batch = local_batch * world
        if len(self.src) < self.global_batch:
            raise ValueError(f"{path}: {len(self.src)} pairs, fewer than one global batch "
                             f"({self.global_batch})")
        self.seed, self.shuffle_buffer, self.shuffle = seed, shuffle_buffer, shuffle
        self.bucket, self.max_len = max(1, int(bucket)), max_len
        self.pin = pin and torch.cuda.is_available()
        # full global batches per epoch (the tail that does not fill one is skipped
        # so every rank runs the same number of synchronous steps)
        self.steps_per_epoch = len(self.src) // self.global_batch
        self._order_epoch = -1
        self._order: List[int] = []
        self._next = 0

    def __len__(self) -> int:
        return len(self.src)

    def _epoch_order(self, epoch: int) -> List[int]:
        if epoch != self._order_epoch:
            n = len(self.src)
            self._order = (buffered_shuffle(n, self.shuffle_buffer, self.seed * 1_000_003 + epoch)
                           if self.shuffle else list(range(n)))
            self._order_epoch = epoch
        return self._order

    def batch(self, step: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """This rank's slice of global batch `step` (epochs wrap around);
        padded to the longest sequence of the whole global batch."""
        epoch, i = divmod(step, self.steps_per_epoch)
        order = self._epoch_order(epoch)
        g = order[i * self.global_batch:(i + 1) * self.global_batch]
        S, T = bucket_lengths(max(len(self.src[j]) for j in g), max(len(self.tgt[j]) for j in g),
                              self.bucket, self.max_len)
        mine = g[self.rank * self.local_batch:(self.rank + 1) * self.local_batch]
        src = pad_rows([self.src[j] for j in mine], S)
        tgt = pad_rows([self.tgt[j] for j in mine], T)
        if self.pin:
            src, tgt = src.pin_memory(), tgt.pin_memory()
        return src, tgt

    def next(self, out=None):
        b = self.batch(self._next)
        self._next += 1
        return b

    def seek(self, step: int) -> None:
        self._next = int(step)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        while True:
            yield self.next()
