"""GDCN reranker input (reference utils/data_preprocessing/feature_processor.py).

Host side keeps the reference's surface (same class / function names, argument meaning and
outputs): FeatureProcessor (:26-111: sklearn StandardScaler over the dense columns, raw log
values kept for the cross features), UserTowerDataset (:116-141), RerankerDataset (:143-181)
and reranker_collate_fn (:184-191). The MI355X path is RerankerBatchBuilder: the feature
tables live in HBM (scaled fp32, raw float64, CSR sequences) and a whole batch of (user, item)
pairs is assembled by rsx_reranker_batch in two launches instead of B __getitem__ calls (each a
pandas .loc per table) plus a host collate and an H2D copy. Its outputs are bit-identical to
reranker_collate_fn over RerankerDataset items (tests/test_gpu_reranker_batch.py).
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch
from sklearn.preprocessing import StandardScaler
from torch.nn.utils.rnn import pad_sequence
from torch.utils.data import Dataset

U_DENSE_COLS = ["user_avg_price_log", "total_cnt_log", "recency_log"]
I_DENSE_COLS = ["pop_1w_log", "pop_1m_log", "velocity_1w", "velocity_1m", "days_since_release_log",
                "avg_item_price_log"]


def _frame(src, index_col):
    return (pd.read_parquet(src) if isinstance(src, str) else src.reset_index() if src.index.name == index_col
            else src).set_index(index_col)


class FeatureProcessor:
    """users / items / seqs: parquet paths (as the reference) or DataFrames holding the same
    columns (customer_id / article_id index or column)."""

    def __init__(self, user_path, item_path, seq_path):
        self.users = _frame(user_path, "customer_id")
        self.items = _frame(item_path, "article_id")
        self.seqs = _frame(seq_path, "customer_id")
        self.u_dense_cols = list(U_DENSE_COLS)
        self.i_dense_cols = list(I_DENSE_COLS)
        # scaled copies for the model inputs; the raw log values stay for the cross features
        self.user_scaler = StandardScaler()
        self.item_scaler = StandardScaler()
        self.users_scaled = self.users.copy()
        self.users_scaled[self.u_dense_cols] = self.user_scaler.fit_transform(self.users[self.u_dense_cols])
        self.items_scaled = self.items.copy()  # raw_probability is not scaled
        self.items_scaled[self.i_dense_cols] = self.item_scaler.fit_transform(self.items[self.i_dense_cols])
        self._tables = {}

    # ---- the reference's per-call accessors (:70-111)
    def get_user_tensor(self, user_ids):
        rows = self.users_scaled.loc[user_ids]
        dense = torch.tensor(rows[self.u_dense_cols].values, dtype=torch.float32)
        cat = torch.tensor(rows["preferred_channel"].values - 1, dtype=torch.long)  # channels 1, 2 -> 0, 1
        return dense, cat

    def get_item_tensor(self, item_ids):
        return torch.tensor(self.items_scaled.loc[item_ids][self.i_dense_cols].values, dtype=torch.float32)

    def get_raw_probability(self, item_ids):
        return torch.tensor(self.items.loc[item_ids]["raw_probability"].values, dtype=torch.float32)

    def get_cross_features(self, user_ids, item_ids):
        """[B, 3] from the unscaled log values: price gap and the two trend interactions."""
        u = self.users.loc[user_ids]
        i = self.items.loc[item_ids]
        gap = i["avg_item_price_log"].values - u["user_avg_price_log"].values
        t1w = i["velocity_1w"].values * u["total_cnt_log"].values
        t1m = i["velocity_1m"].values * u["total_cnt_log"].values
        return torch.tensor(np.stack([gap, t1w, t1m], axis=1), dtype=torch.float32)

    # ---- device tables for RerankerBatchBuilder
    def device_tables(self, device):
        """HBM-resident tables in users / items row order (cached per device)."""
        key = str(torch.device(device))
        if key in self._tables:
            return self._tables[key]
        dev = torch.device(device)
        seq_col = self.seqs["sequence_ids"].reindex(self.users.index)
        lens = np.array([0 if not isinstance(s, (list, np.ndarray)) else len(s) for s in seq_col], dtype=np.int64)
        off = np.zeros(len(lens) + 1, dtype=np.int64)
        np.cumsum(lens, out=off[1:])
        flat = (np.concatenate([np.asarray(s, dtype=np.int64) for s in seq_col if isinstance(s, (list, np.ndarray))
                                and len(s)]) if off[-1] else np.zeros(1, dtype=np.int64))
        item_num = np.array([int(s) if str(s).isdigit() else 0 for s in self.items.index.astype(str)], dtype=np.int64)
        t = {
            "u_scaled": torch.tensor(self.users_scaled[self.u_dense_cols].values, dtype=torch.float32),
            "u_raw": torch.tensor(self.users[["user_avg_price_log", "total_cnt_log"]].values, dtype=torch.float64),
            "u_cat": torch.tensor(self.users["preferred_channel"].values - 1, dtype=torch.int64),
            "i_scaled": torch.tensor(self.items_scaled[self.i_dense_cols].values, dtype=torch.float32),
            "i_raw": torch.tensor(self.items[["avg_item_price_log", "velocity_1w", "velocity_1m"]].values,
                                  dtype=torch.float64),
            "i_num": torch.from_numpy(item_num),
            "seq_off": torch.from_numpy(off),
            "seq_ids": torch.from_numpy(flat),
        }
        t = {k: v.contiguous().to(dev) for k, v in t.items()}
        self._tables[key] = t
        return t


class UserTowerDataset(Dataset):
    """Per-user inputs of the user tower (:116-141)."""

    def __init__(self, user_ids, processor, max_seq_len=50):
        self.user_ids = user_ids
        self.processor = processor
        self.max_len = max_seq_len

    def __len__(self):
        return len(self.user_ids)

    def __getitem__(self, idx):
        uid = self.user_ids[idx]
        dense, cat = self.processor.get_user_tensor([uid])
        if uid in self.processor.seqs.index:
            row = self.processor.seqs.loc[uid]
            ids, deltas = row["sequence_ids"][-self.max_len:], row["sequence_deltas"][-self.max_len:]
        else:  # users without a sequence
            ids, deltas = [], []
        return {"user_dense": dense.squeeze(0), "user_cat": cat.squeeze(0),
                "seq_ids": torch.tensor(ids, dtype=torch.long), "seq_deltas": torch.tensor(deltas, dtype=torch.long)}


class RerankerDataset(Dataset):
    """One (user, item, label) interaction -> the GDCN input (:143-181): 12 dense features
    (user 3 scaled | item 6 scaled | 3 cross), the user's channel, the last max_seq_len
    sequence ids, the numeric target item id and the label."""

    def __init__(self, interactions_df, processor, max_seq_len=50):
        self.data = interactions_df
        self.processor = processor
        self.max_len = max_seq_len

    def __len__(self):
        return len(self.data)

    def __getitem__(self, idx):
        row = self.data.iloc[idx]
        uid, iid = str(row["user_id"]), str(row["item_id"])
        u_dense, u_cat = self.processor.get_user_tensor([uid])
        i_dense = self.processor.get_item_tensor([iid])
        cross = self.processor.get_cross_features([uid], [iid])
        dense = torch.cat([u_dense.squeeze(0), i_dense.squeeze(0), cross.squeeze(0)], dim=0)
        if uid in self.processor.seqs.index:
            seq = torch.tensor(self.processor.seqs.loc[uid]["sequence_ids"][-self.max_len:], dtype=torch.long)
        else:
            seq = torch.tensor([], dtype=torch.long)
        return {"gdcn_dense": dense, "user_cat": u_cat.squeeze(0), "seq_ids": seq,
                "target_item_id": torch.tensor(int(iid) if iid.isdigit() else 0),
                "label": torch.tensor(row["label"], dtype=torch.float32)}


def reranker_collate_fn(batch):
    """(dense [B,12], cat [B], seq_ids [B,L] right-padded with 0, seq_mask, target [B], label [B])."""
    dense = torch.stack([b["gdcn_dense"] for b in batch])
    cat = torch.stack([b["user_cat"] for b in batch])
    label = torch.stack([b["label"] for b in batch])
    target = torch.stack([b["target_item_id"] for b in batch])
    seq = pad_sequence([b["seq_ids"] for b in batch], batch_first=True, padding_value=0)
    return dense, cat, seq, (seq != 0).long(), target, label


class RerankerBatchBuilder:
    """Device-side RerankerDataset + reranker_collate_fn: build(user_ids, item_ids, labels)
    returns the collate tuple on `device`, assembled by rsx_reranker_batch from the processor's
    HBM tables. Unknown ids raise KeyError (the reference's .loc does)."""

    def __init__(self, processor, device, max_seq_len=50):
        self.processor = processor
        self.device = torch.device(device)
        self.max_len = int(max_seq_len)
        self.tables = processor.device_tables(self.device)

    def rows(self, user_ids, item_ids):
        u = self.processor.users.index.get_indexer([str(x) for x in user_ids])
        i = self.processor.items.index.get_indexer([str(x) for x in item_ids])
        if (u < 0).any() or (i < 0).any():
            missing = [x for x, r in zip(user_ids, u) if r < 0] + [x for x, r in zip(item_ids, i) if r < 0]
            raise KeyError(f"unknown ids: {missing[:5]}")
        return (torch.from_numpy(u.astype(np.int64)).to(self.device),
                torch.from_numpy(i.astype(np.int64)).to(self.device))

    def build(self, user_ids, item_ids, labels):
        from ... import ops
        uidx, iidx = self.rows(user_ids, item_ids)
        dense, cat, seq, mask, target = ops.reranker_batch(uidx, iidx, self.tables, self.max_len)
        label = torch.as_tensor(np.asarray(labels), dtype=torch.float32).to(self.device)
        return dense, cat, seq, mask, target, label

    def from_interactions(self, interactions_df):
        return self.build(interactions_df["user_id"].tolist(), interactions_df["item_id"].tolist(),
                          interactions_df["label"].tolist())
