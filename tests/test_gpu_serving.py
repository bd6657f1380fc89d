"""The serving endpoints end to end on the GPU: refresh-item-vectors (batched eval forward of
HybridItemTower, files in the reference's format) and train/item-tower (SimCSE epochs)."""
import os

import pytest
import torch

import recsys_amd  # noqa: F401
from recsys_amd import item_data as D
from recsys_amd import item_tower as IT

pytestmark = pytest.mark.gpu


@pytest.fixture()
def app_client(gpu, tmp_path):
    from fastapi import FastAPI
    from fastapi.testclient import TestClient
    from recsys_amd.APIController import serving_controller as SC
    from recsys_amd.utils import dependencies as deps
    torch.manual_seed(0)
    bert = IT.build_local_bert(hidden_size=64, num_layers=2, num_heads=4, intermediate=128, seed=1)
    deps.initialize_global_models(384, 6, 128, bert_model=bert, batch_size=8, device=gpu)
    deps.set_product_store(D.InMemoryProductStore(D.synthetic_product_rows(37, seed=3)))
    SC.MODEL_DIR = str(tmp_path / "ckpt")
    app = FastAPI()
    app.include_router(SC.serving_controller_router, prefix="/ai-api/serving")
    yield TestClient(app), deps, tmp_path
    deps.set_product_store(D.InMemoryProductStore())
    deps.global_encoder = deps.global_projector = None


def test_refresh_item_vectors_endpoint(app_client):
    client, deps, tmp = app_client
    r = client.post("/ai-api/serving/bg/inference/refresh-item-vectors", params={"save_dir": str(tmp / "m")})
    assert r.status_code == 200, r.text
    body = r.json()
    assert body["item_count"] == 37 and body["vector_shape"] == [37, 128]
    mat = torch.load(body["saved_path_matrix"], weights_only=True)
    ids = torch.load(body["saved_path_ids"], weights_only=True)
    assert ids == sorted(str(i) for i in range(1, 38))
    assert torch.allclose(mat.norm(dim=1), torch.ones(37), atol=1e-5)
    # the same vectors as one direct eval forward over the whole (id-sorted, tagged) set
    rows = deps.global_product_store.fetch_products()
    items = sorted((D.parse_db_row(x) for x in rows), key=lambda x: x.product_id)
    col = D.SimCSECollator()                       # the fixed reference vocabulary
    enc = deps.get_global_encoder().eval()
    with torch.no_grad():
        ref = enc(*[t.cuda() for t in col.process_batch_items(items)]).cpu()
    torch.testing.assert_close(mat, ref, atol=1e-4, rtol=1e-4)


def test_train_item_tower_endpoint(app_client):
    client, deps, tmp = app_client
    before = {k: v.clone() for k, v in deps.get_global_projector().state_dict().items()}
    r = client.post("/ai-api/serving/train/item-tower", params={"epochs": 1, "lr": 1e-3})
    assert r.status_code == 200, r.text
    losses = r.json()["epoch_avg_loss"]
    assert len(losses) == 1 and losses[0] == losses[0] and losses[0] > 0
    after = deps.get_global_projector().state_dict()
    assert any(not torch.equal(before[k], after[k]) for k in before)
    ck = os.listdir(tmp / "ckpt")
    assert len(ck) == 1 and ck[0].startswith("encoder_ep01_loss")
    missing = client.post("/ai-api/serving/bg/inference/refresh-item-vectors",
                          params={"save_dir": str(tmp / "m2"), "checkpoint_path": str(tmp / "nope.pth")})
    assert missing.status_code == 500
    ok = client.post("/ai-api/serving/bg/inference/refresh-item-vectors",
                     params={"save_dir": str(tmp / "m3"), "checkpoint_path": str(tmp / "ckpt" / ck[0])})
    assert ok.status_code == 200, ok.text


def test_similarity_endpoint_exact_top50(gpu):
    """GET /similarity/pgvector/{id} on the GPU index: the 50 nearest other items by exact cosine
    (the reference asks pgvector's approximate HNSW), in the reference's response shape."""
    from fastapi import FastAPI
    from fastapi.testclient import TestClient
    from recsys_amd.APIController import controller as C
    g = torch.Generator().manual_seed(5)
    ids = list(range(1000, 1000 + 3000))
    vecs = torch.randn(3000, 128, generator=g)
    C.set_vector_index(C.ItemVectorIndex(ids, vecs, {i: f"cat{i % 7}" for i in ids}, device=gpu))
    app = FastAPI()
    app.include_router(C.controller_router, prefix="/ai-api/controller")
    cl = TestClient(app)
    try:
        r = cl.get("/ai-api/controller/similarity/pgvector/1234")
        assert r.status_code == 200, r.text
        body = r.json()
        hits = body["top_5_similar"]
        assert len(hits) == 50 and body["query_item"] == {"id": 1234, "category": "cat2"}
        vn = torch.nn.functional.normalize(vecs.double(), dim=1)
        sim = vn @ vn[234]
        sim[234] = -2
        ref = torch.argsort(-sim, stable=True)[:50]
        assert [h["id"] for h in hits] == [ids[int(i)] for i in ref]
        assert abs(hits[0]["rank_score"] - round(float(sim[ref[0]]), 4)) < 1e-4
        assert abs(hits[0]["raw_distance"] - round(1 - float(sim[ref[0]]), 4)) < 1e-4
        assert cl.get("/ai-api/controller/similarity/pgvector/7").status_code == 404
    finally:
        C.set_vector_index(None)
