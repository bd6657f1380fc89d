"""CPU restatement of the user-side input producer -- TEST INFRASTRUCTURE ONLY.

Pure-Python loops (the reference's own control flow, one customer at a time):
  * sequences_from_transactions: staticstics/preprosess_agg_parallel.py:410-431
    (process_sequence_row: purchases ordered by day, the last 50 kept, delta = last day - day)
    with days_int = days since 1970-01-01 (:452). The reference orders by
    sort_values('days_int') (quicksort); same-day purchases keep their input order here (a
    stable sort) -- the reference's committed sample is already date-sorted, so this is its
    file order.
  * lookup_arrays: tower_code/v1_refine_usertower.py:55-122 (FeatureProcessor id maps and the
    fast lookup arrays, filled row by row as the reference's iterrows loops do).
  * sample: tower_code/v1_refine_usertower.py:204-306 (SASRecDataset.__getitem__).
Parity is pinned by the reference's own data file (staticstics/customer_sample_view.json, a
slice committed under tests/golden/); no reference code is imported.
"""
import datetime

BINS = [0, 3, 7, 14, 30, 60, 180, 330, 395]


def digitize(x):
    """np.digitize(x, BINS, right=False): the number of bins <= x (0 below the first edge)."""
    n = 0
    for b in BINS:
        if x >= b:
            n += 1
    return n


def _days(date_str):
    d = datetime.date.fromisoformat(date_str)
    return (d - datetime.date(1970, 1, 1)).days


def sequences_from_transactions(rows, cap=50):
    """rows: [{'customer_id', 'article_id': [...], 't_dat': ['YYYY-MM-DD', ...]}] ->
    {customer_id: (sequence_ids, sequence_deltas)} (preprosess_agg_parallel.py:410-431)."""
    out = {}
    for r in rows:
        days = [_days(t) for t in r["t_dat"]]
        order = sorted(range(len(days)), key=lambda i: days[i])
        arts = [r["article_id"][i] for i in order]
        ds = [days[i] for i in order]
        if len(arts) > cap:
            arts, ds = arts[-cap:], ds[-cap:]
        last = ds[-1]
        out[r["customer_id"]] = (arts, [last - d for d in ds])
    return out


def lookup_arrays(user_rows, item_rows, user_order, item_order):
    """FeatureProcessor (v1_refine_usertower.py:55-122) on plain dicts: user_rows[uid] / item_rows[iid]
    are dicts of the frame columns; user_order / item_order the frames' row order.
    -> (user2id, item2id, u_bucket, u_cat, u_cont, i_side) as lists of lists."""
    user2id = {uid: i + 1 for i, uid in enumerate(user_order)}
    item2id = {iid: i + 1 for i, iid in enumerate(item_order)}
    nu = len(user_order) + 1
    u_bucket = [[0] * 4 for _ in range(nu)]
    u_cat = [[0] * 5 for _ in range(nu)]
    u_cont = [[0.0] * 4 for _ in range(nu)]
    for uid in user_order:
        row = user_rows[uid]
        k = user2id[uid]
        u_bucket[k] = [int(row["age_bucket"]), int(row["user_avg_price_bucket"]), int(row["total_cnt_bucket"]),
                       int(row["recency_bucket"])]
        u_cat[k] = [int(row["preferred_channel"]), int(row["club_member_status_idx"]),
                    int(row["fashion_news_frequency_idx"]), int(row["FN"]), int(row["Active"])]
        u_cont[k] = [float(row["price_std_scaled"]), float(row["last_price_diff_scaled"]),
                     float(row["repurchase_ratio_scaled"]), float(row["weekend_ratio_scaled"])]
    i_side = [[0] * 4 for _ in range(len(item_order) + 1)]
    for iid in item_order:
        row = item_rows[iid]
        i_side[item2id[iid]] = [int(row.get(c, 0)) for c in ("type_id", "color_id", "graphic_id", "section_id")]
    return user2id, item2id, u_bucket, u_cat, u_cont, i_side


def sample(user_id, seq_ids, seq_deltas, arrays, max_len, is_train):
    """SASRecDataset.__getitem__ (v1_refine_usertower.py:204-306) -> dict of plain lists / scalars."""
    user2id, item2id, u_bucket, u_cat, u_cont, i_side = arrays
    u = user2id.get(user_id, 0)
    tb = [digitize(d) for d in seq_deltas]
    seq = [item2id.get(it, 0) for it in seq_ids]
    if is_train:
        seq = seq[-(max_len + 1):]
        tb = tb[-(max_len + 1):]
        if len(seq) > 1:
            inp, tgt, tin = seq[:-1], seq[1:], tb[:-1]
        else:
            inp, tgt, tin = seq, seq, tb
    else:
        inp, tgt, tin = seq[-max_len:], [], tb[-max_len:]
    pad = max_len - len(inp)
    item = [0] * pad + inp
    time_ = [0] * pad + tin
    target = [0] * pad + tgt if is_train else [0] * max_len
    side = [i_side[i] for i in item]
    return {"user_ids": user_id, "item_ids": item, "target_ids": target,
            "padding_mask": [True] * pad + [False] * len(inp), "time_bucket_ids": time_,
            "type_ids": [s[0] for s in side], "color_ids": [s[1] for s in side],
            "graphic_ids": [s[2] for s in side], "section_ids": [s[3] for s in side],
            "age_bucket": u_bucket[u][0], "price_bucket": u_bucket[u][1], "cnt_bucket": u_bucket[u][2],
            "recency_bucket": u_bucket[u][3], "channel_ids": u_cat[u][0], "club_status_ids": u_cat[u][1],
            "news_freq_ids": u_cat[u][2], "fn_ids": u_cat[u][3], "active_ids": u_cat[u][4],
            "cont_feats": list(u_cont[u])}
