"""Drop-in for utils/vocab.py: the fixed STD vocabulary of the item tower's input contract.

Reference (restated): ``STD_VOCAB_CONFIG`` :5-418 (6 fields of H&M values, 399 entries, 382
distinct), ``RE_FEATURE_KEYS`` :421-424, ``PAD_ID = 0`` / ``UNK_ID = 1`` :427-428, the merged
vocabulary ``ALL_STD_TOKENS = sorted(set(...))`` with ``id = 2 + index`` :431-434, and the
helpers :436-444 (``get_std_vocab_size() == 384``).

The table itself is data: ``std_vocab.json`` next to this file, regenerated from the reference
text by ``tools/make_std_vocab.py`` (field order and value order preserved). Ids are therefore
the reference's ids, identical in training (item_tower.train_simcse_from_db) and in the
item-vector refresh (utils/inference_utils.py), independent of which products are at hand.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List

_HERE = os.path.dirname(os.path.abspath(__file__))

with open(os.path.join(_HERE, "std_vocab.json"), encoding="utf-8") as _f:
    _DOC = json.load(_f)

STD_VOCAB_CONFIG: Dict[str, List[str]] = {fd["key"]: list(fd["values"]) for fd in _DOC["fields"]}

RE_FEATURE_KEYS = ["[CAT]", "[MAT]", "[DET]", "[FIT]", "[FNC]", "[SPC]", "[COL]", "[CTX]", "[LOC]"]

PAD_ID = 0
UNK_ID = 1

ALL_STD_TOKENS: List[str] = sorted({tok for vals in STD_VOCAB_CONFIG.values() for tok in vals})
STD_TOKEN_TO_ID: Dict[str, int] = {tok: i + 2 for i, tok in enumerate(ALL_STD_TOKENS)}


def get_std_vocab_size() -> int:
    """:436-437 — distinct tokens + PAD + UNK (384)."""
    return len(STD_TOKEN_TO_ID) + 2


def get_std_id(value) -> int:
    """:439-441 — empty/None -> PAD, unknown -> UNK, else 2 + sorted index."""
    if not value:
        return PAD_ID
    return STD_TOKEN_TO_ID.get(str(value), UNK_ID)


def get_std_field_keys() -> List[str]:
    """:443-444 — the six STD fields in the table's order."""
    return list(STD_VOCAB_CONFIG.keys())
