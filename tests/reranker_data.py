"""Seeded H&M-shaped feature tables for the reranker-input tests (users / items / sequences,
the columns utils/data_preprocessing/feature_processor.py reads)."""
import numpy as np
import pandas as pd


def make_tables(n_users=400, n_items=300, seed=0):
    rng = np.random.default_rng(seed)
    uids = [f"{rng.integers(0, 2**63):016x}" for _ in range(n_users)]
    users = pd.DataFrame({
        "customer_id": uids,
        "user_avg_price_log": rng.normal(-3.5, 0.6, n_users),
        "total_cnt_log": np.log1p(rng.integers(1, 400, n_users)).astype(np.float64),
        "recency_log": np.log1p(rng.integers(0, 700, n_users)).astype(np.float64),
        "preferred_channel": rng.integers(1, 3, n_users),
    })
    iids = [f"0{rng.integers(100000000, 999999999)}" for _ in range(n_items)]
    iids[3] = "A12345"  # not all digits -> target id 0
    items = pd.DataFrame({
        "article_id": iids,
        "pop_1w_log": rng.normal(2.0, 1.0, n_items),
        "pop_1m_log": rng.normal(3.0, 1.2, n_items),
        "velocity_1w": rng.normal(0.5, 1.0, n_items),
        "velocity_1m": rng.normal(0.2, 0.8, n_items),
        "days_since_release_log": np.log1p(rng.integers(0, 900, n_items)).astype(np.float64),
        "avg_item_price_log": rng.normal(-3.4, 0.5, n_items),
        "raw_probability": rng.random(n_items),
    })
    items.loc[7, "pop_1w_log"] = 2.0  # keep a constant-free column set; one exact value repeat
    has_seq = rng.random(n_users) < 0.85
    seq_ids, seq_deltas, seq_users = [], [], []
    for u, ok in zip(uids, has_seq):
        if not ok:
            continue
        n = int(rng.integers(0, 120))  # some longer than the 50-step window, some empty
        ids = rng.integers(1, 47063, n)
        if n > 5 and rng.random() < 0.2:
            ids[rng.integers(0, n)] = 0  # an unknown item mapped to 0 inside a sequence (masked)
        seq_users.append(u)
        seq_ids.append(ids.tolist())
        seq_deltas.append(rng.integers(1, 10, n).tolist())
    seqs = pd.DataFrame({"customer_id": seq_users, "sequence_ids": seq_ids, "sequence_deltas": seq_deltas})
    return users.set_index("customer_id"), items.set_index("article_id"), seqs.set_index("customer_id")


def interactions(users, items, n=96, seed=1):
    rng = np.random.default_rng(seed)
    return pd.DataFrame({"user_id": rng.choice(users.index.values, n), "item_id": rng.choice(items.index.values, n),
                         "label": rng.integers(0, 2, n)})
