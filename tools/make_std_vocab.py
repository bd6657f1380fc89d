"""Regenerates utils/std_vocab.json: the reference's fixed STD vocabulary table
(/root/reference/utils/vocab.py:5-418, ``STD_VOCAB_CONFIG``) as data.

The reference file is parsed as text (``ast`` + ``literal_eval`` of the one dict literal);
nothing from it is imported or executed. Only this container has /root/reference; the JSON
is committed so the package and the GPU box never read the reference.

  python tools/make_std_vocab.py [/root/reference/utils/vocab.py]
"""
import ast
import json
import os
import sys

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/utils/vocab.py"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "llm-driven_content-based-feature_recommendation_system_amd", "utils", "std_vocab.json")

tree = ast.parse(open(SRC, encoding="utf-8").read())
table = None
for node in tree.body:
    if isinstance(node, ast.Assign) and getattr(node.targets[0], "id", "") == "STD_VOCAB_CONFIG":
        table = ast.literal_eval(node.value)
assert table is not None, "STD_VOCAB_CONFIG not found"
doc = {"source": "utils/vocab.py:5-418 (STD_VOCAB_CONFIG), field order and value order as in the reference",
       "fields": [{"key": k, "values": list(v)} for k, v in table.items()]}
with open(OUT, "w", encoding="utf-8") as f:
    f.write('{"source": %s,\n "fields": [\n' % json.dumps(doc["source"]))
    f.write(",\n".join("  " + json.dumps(fd, ensure_ascii=False) for fd in doc["fields"]))
    f.write("\n]}\n")
print(OUT, sum(len(v) for v in table.values()), "values,", len({x for v in table.values() for x in v}), "distinct")
