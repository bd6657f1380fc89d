"""refresh-item-vectors forward (bench.py's bench_item_refresh shape: 768 products, bert-base
BERT, text lengths U{2..32}) with the packed-token BERT and with HF BertModel (the packing
check forced off). Prints items/s of each.  python tools/refresh_micro.py"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import recsys_amd  # noqa: E402,F401
from recsys_amd import item_tower as IT  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    args = argparse.Namespace(seed=0)
    res = {"packed": bench.bench_item_refresh(args, dev)}
    ok = IT.bert_packed_ok
    IT.bert_packed_ok = lambda *a: False
    res["bertmodel"] = bench.bench_item_refresh(args, dev)
    IT.bert_packed_ok = ok
    print(json.dumps({k: {"items_per_s": v["value"], "ms_per_batch": v["ms_per_batch"]} for k, v in res.items()}),
          flush=True)


if __name__ == "__main__":
    main()
