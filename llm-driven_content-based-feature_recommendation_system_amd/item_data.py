"""Host-side data contract of the item tower: products -> (std, re_ids, re_mask, txt_ids,
txt_mask) tensors, the SimCSE two-view corruption, and the product source the serving
endpoints read.

Reference (restated, not imported):
  * TrainingItem                      database.py:40-43
  * SimCSERecSysDataset._corrupt_data item_tower.py:341-394 (two corrupted views per product)
  * SimCSECollator.process_batch_items item_tower.py:505-597 (STD ids, "prompt: value" RE
    fields tokenised to MAX_RE_LEN, product name tokenised to MAX_TXT_LEN)
  * FIELD_PROMPT_MAP / MAX_RE_LEN / MAX_TXT_LEN item_tower.py:448-463
  * RE_FEATURE_KEYS, PAD/UNK ids, STD id = 2 + sorted-token index  utils/vocab.py:421-444
  * ProductInferenceInput rows (product_id, feature_data, product_name) database.py:58-70

This is host ETL (SURVEY.md §2 marks the tokenizer/collator out of the GPU scope); it exists so
the drop-in endpoints (APIController/serving_controller.py) run end to end offline:
  * the reference tokenises with ``bert-base-uncased`` fetched by name; offline there is no
    vocabulary file, so the default ``HashingTokenizer`` maps lower-cased words to ids in
    [1000, vocab) by a fixed hash with BERT's special ids (CLS 101, SEP 102, PAD 0). Pass any
    callable with the HF tokenizer's ``(text, max_length) -> (ids, mask)`` contract instead;
  * the STD vocabulary is the reference's fixed table (utils/vocab.py here, restated from
    utils/vocab.py:5-444: 382 values, ids 2..383, PAD 0, UNK 1), the collator's default;
  * the product source is any object with ``fetch_products() -> list[dict]`` (the rows of
    ``select(ProductInferenceInput.product_id, .feature_data, .product_name)``); a maintainer
    adapts a SQLAlchemy session with a three-line wrapper.
"""
from __future__ import annotations

import copy
import random
import zlib
from typing import Any, Dict, Iterable, List, Optional, Sequence

import torch
from pydantic import BaseModel

from .utils.vocab import (PAD_ID, RE_FEATURE_KEYS, STD_TOKEN_TO_ID, STD_VOCAB_CONFIG, UNK_ID,  # noqa: F401
                          get_std_field_keys, get_std_vocab_size)

CLS_ID, SEP_ID = 101, 102          # bert-base-uncased special ids
STD_FIELD_KEYS = get_std_field_keys()
FIELD_PROMPT_MAP = {"[CAT]": "Clothing Category", "[MAT]": "Fabric Material", "[DET]": "Garment Detail",
                    "[FIT]": "Clothing Fit", "[FNC]": "Apparel Function", "[SPC]": "Product Specification",
                    "[COL]": "Garment Color", "[CTX]": "Occasion", "[LOC]": "Body Part"}
MAX_RE_LEN = 32
MAX_TXT_LEN = 32


class TrainingItem(BaseModel):
    """database.py:40-43."""
    product_id: str
    feature_data: Dict[str, Any]
    product_name: str


def flatten_reinforced(raw: Dict[str, Any]) -> Dict[str, Any]:
    """train_simcse_from_db :904-918: 'reinforced_feature' sub-dict keys become "[KEY]" fields."""
    feats = dict(raw)
    re_dict = feats.get("reinforced_feature")
    if isinstance(re_dict, dict):
        for key, val in re_dict.items():
            feats[key if key.startswith("[") and key.endswith("]") else f"[{key}]"] = val
    return feats


def parse_db_row(row: Dict[str, Any]) -> TrainingItem:
    """utils/inference_utils.py:13-50 (the inference-side row parser): flattened RE fields and
    the TAGGED name "<name> (Category: <type>)", or "<type> <appearance>" / "Unknown Product"
    when the name is empty (training uses the raw name instead: SURVEY.md Appendix B #8)."""
    feats = flatten_reinforced(row["feature_data"] or {})
    base = row.get("product_name")
    ptype = str(feats.get("product_type_name", "")).strip()
    if base:
        name = f"{base} (Category: {ptype})" if ptype else base
    else:
        name = f"{ptype} {str(feats.get('graphical_appearance_name', '')).strip()}".strip() or "Unknown Product"
    return TrainingItem(product_id=str(row["product_id"]), feature_data=feats, product_name=name)


def rows_to_items(rows: Iterable[Dict[str, Any]]) -> List[TrainingItem]:
    """DB rows -> TrainingItems (train_simcse_from_db :898-950, parse_db_row)."""
    return [TrainingItem(product_id=str(r["product_id"]), feature_data=flatten_reinforced(r["feature_data"] or {}),
                         product_name=r.get("product_name") or "") for r in rows]


class InMemoryProductStore:
    """The product source the endpoints use when no database is wired: a list of rows with
    the ProductInferenceInput columns. ``fetch_products()`` returns them sorted by id."""

    def __init__(self, rows: Sequence[Dict[str, Any]] = ()):
        self.rows = [dict(r) for r in rows]

    def fetch_products(self) -> List[Dict[str, Any]]:
        return sorted(self.rows, key=lambda r: int(r["product_id"]))


class HashingTokenizer:
    """Offline stand-in for the bert-base-uncased tokenizer call the collator makes
    (``padding='max_length', truncation=True, add_special_tokens=True``): [CLS] w1 .. wn [SEP]
    then PAD, mask 1 on the non-pad positions. Word ids: crc32(lower-cased word) mapped into
    [1000, vocab_size). "[SEP]" in the text becomes SEP_ID (the collator joins list values
    with it, item_tower.py:485-500)."""

    sep_token = "[SEP]"

    def __init__(self, vocab_size: int = 30522):
        self.vocab_size = vocab_size

    def word_id(self, w: str) -> int:
        if w == self.sep_token:
            return SEP_ID
        return 1000 + zlib.crc32(w.lower().encode()) % (self.vocab_size - 1000)

    def __call__(self, text: str, max_length: int):
        ids = [CLS_ID] + [self.word_id(w) for w in text.split()][: max_length - 2] + [SEP_ID]
        mask = [1] * len(ids)
        pad = max_length - len(ids)
        return ids + [PAD_ID] * pad, mask + [0] * pad


class SimCSECollator:
    """item_tower.py:465-605 with an injectable tokenizer. The STD vocabulary defaults to the
    reference's fixed table (utils/vocab.py: ids 2..383, ``std_vocab_size`` 384); an injected
    one must keep every id below ``std_vocab_size`` (the embedding's row count): checked here,
    on the host, before any tensor reaches the GPU gather."""

    def __init__(self, tokenizer=None, std_vocab: Optional[Dict[str, int]] = None,
                 std_keys: Sequence[str] = STD_FIELD_KEYS, max_re_len: int = MAX_RE_LEN,
                 max_txt_len: int = MAX_TXT_LEN, std_vocab_size: Optional[int] = None):
        self.tokenizer = tokenizer or HashingTokenizer()
        self.std_vocab = STD_TOKEN_TO_ID if std_vocab is None else std_vocab
        self.std_vocab_size = get_std_vocab_size() if std_vocab_size is None else int(std_vocab_size)
        top = max(self.std_vocab.values(), default=UNK_ID)
        if top >= self.std_vocab_size or min(self.std_vocab.values(), default=2) < 0:
            raise ValueError(f"STD vocabulary ids must lie in [0, {self.std_vocab_size}); got max id {top}")
        self.std_keys = list(std_keys)
        self.re_keys = RE_FEATURE_KEYS
        self.max_re_len = max_re_len
        self.max_txt_len = max_txt_len
        self.sep = getattr(self.tokenizer, "sep_token", "[SEP]")

    def std_id(self, value) -> int:
        """utils/vocab.py:439-441."""
        if not value:
            return PAD_ID
        return self.std_vocab.get(str(value), UNK_ID)

    def _serialize(self, value: Any) -> str:
        """item_tower.py:485-500: lists joined with ' [SEP] '."""
        if not value:
            return ""
        if isinstance(value, list):
            vals = [str(v) for v in value if v]
            return f" {self.sep} ".join(vals) if vals else ""
        return str(value)

    def process_batch_items(self, items: List[TrainingItem], is_first_view: bool = False):
        """-> (std [B,F], re_ids [B,9,R], re_mask [B,9,R], txt_ids [B,S], txt_mask [B,S]) int64."""
        std, re_ids, re_mask, txt_ids, txt_mask = [], [], [], [], []
        for it in items:
            std.append([self.std_id(it.feature_data.get(k, "")) for k in self.std_keys])
            ids_i, mask_i = [], []
            for key in self.re_keys:
                val = self._serialize(it.feature_data.get(key))
                text = f"{FIELD_PROMPT_MAP.get(key, key)}: {val}" if val else ""
                ids, mask = self.tokenizer(text, self.max_re_len)
                ids_i.append(ids)
                mask_i.append(mask)
            re_ids.append(ids_i)
            re_mask.append(mask_i)
            ids, mask = self.tokenizer(it.product_name, self.max_txt_len)
            txt_ids.append(ids)
            txt_mask.append(mask)
        t = lambda x: torch.tensor(x, dtype=torch.long)  # noqa: E731
        return t(std), t(re_ids), t(re_mask), t(txt_ids), t(txt_mask)

    def __call__(self, batch):
        v1 = [b[0] for b in batch]
        v2 = [b[1] for b in batch]
        return self.process_batch_items(v1, True), self.process_batch_items(v2, False)


class SimCSERecSysDataset(torch.utils.data.Dataset):
    """item_tower.py:329-463: each product yields two independently corrupted views."""

    def __init__(self, products: List[TrainingItem], dropout_prob: float = 0.2, rng: Optional[random.Random] = None):
        self.products = products
        self.dropout_prob = dropout_prob
        self.rng = rng or random.Random()

    def __len__(self):
        return len(self.products)

    def _corrupt_data(self, item: TrainingItem) -> TrainingItem:
        """:341-394: list values lose each element w.p. p (key dropped if emptied); scalar keys
        dropped w.p. p - 0.1; a multi-word name loses one word w.p. 0.5, a one-word name is
        blanked w.p. 0.1."""
        r = self.rng
        feats = copy.deepcopy(item.feature_data)
        name = item.product_name
        key_p, val_p = self.dropout_prob - 0.1, self.dropout_prob
        for k in list(feats.keys()):
            v = feats[k]
            if isinstance(v, list):
                keep = [x for x in v if r.random() > val_p]
                if keep:
                    feats[k] = keep
                else:
                    del feats[k]
            elif r.random() < key_p:
                del feats[k]
        if name:
            words = name.split()
            if len(words) > 1:
                if r.random() < 0.5:
                    del words[r.randint(0, len(words) - 1)]
                    name = " ".join(words)
            elif r.random() < 0.1:
                name = ""
        return TrainingItem(product_id=item.product_id, feature_data=feats, product_name=name)

    def __getitem__(self, idx):
        it = self.products[idx]
        return self._corrupt_data(it), self._corrupt_data(it)


def synthetic_product_rows(n: int, seed: int = 0) -> List[Dict[str, Any]]:
    """H&M-shaped synthetic products (ids 1..n): the six STD fields drawn from the reference's
    value table (utils/vocab.py; 2 % of values out of vocabulary -> UNK), a few RE list fields
    and a short name. For tests and the offline endpoints."""
    rng = random.Random(seed)
    pools = {k: list(STD_VOCAB_CONFIG[k]) + [f"unlisted {k} {i}" for i in range(2)] for k in STD_FIELD_KEYS}
    words = [f"w{i}" for i in range(400)]
    rows = []
    for pid in range(1, n + 1):
        feats: Dict[str, Any] = {k: rng.choice(pools[k]) for k in STD_FIELD_KEYS if rng.random() > 0.05}
        re = {}
        for key in RE_FEATURE_KEYS:
            if rng.random() < 0.7:
                re[key.strip("[]")] = [" ".join(rng.choices(words, k=rng.randint(1, 4)))
                                       for _ in range(rng.randint(1, 3))]
        feats["reinforced_feature"] = re
        rows.append({"product_id": pid, "feature_data": feats,
                     "product_name": " ".join(rng.choices(words, k=rng.randint(0, 6)))})
    return rows
