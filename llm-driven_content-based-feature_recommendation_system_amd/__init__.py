"""MI355X-native (gfx950) two-tower retrieval + contrastive training + DeepFM rerank path.

Drop-in mirrors of the reference modules live in the sub-packages with the reference's
own names (tower_code, temp_model, APIController, utils, item_tower); the compute runs in
librecsys_amd.so (HIP, C ABI in include/recsys_amd.h) through ops.py.
Import through the alias module `recsys_amd` (the directory name is not an identifier).
"""
__version__ = "0.1.0"
