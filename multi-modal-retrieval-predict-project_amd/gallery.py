"""Gallery build pipeline — the reference's embedding-DB writers on the GPU
towers:

  build_gallery   src/Helpers/contruct_test_db.py:123-142 and src/Trainner/train.py:807-816: run the
                  model over (image, input_ids, attention_mask, record ids) batches, stack the
                  joint embeddings, np.save("<split>_joint_embeddings.npy") (float32 (N, D)) and
                  json.dump(ids, "<split>_ids.json").  Batches are embedded on the device and copied
                  to the host once per batch on a side stream (double-buffered), so the towers of the
                  next batch overlap the device->host copy of the previous one.
  merge_galleries src/Helpers/dumpEmbedding.py:8-42: train + val -> trainval (concatenate rows / ids).

The files are exactly what RetrievalEngine.__init__ (retrieval.py:24-32) loads.  DICOM decoding and
tokenisation (src/DataHandler) stay outside: batches arrive as tensors of the DataLoader contract.
"""
import json
from pathlib import Path
from typing import Iterable, List, Tuple

import numpy as np
import torch


def build_gallery(model, batches: Iterable[Tuple[torch.Tensor, torch.Tensor, torch.Tensor, List[str]]],
                  out_dir, split: str = "test"):
    """-> (embs (N, D) float32 numpy, ids list).  `model` is a MultiModalRetrievalModel (its
    query_embeddings path for multimodal; forward()["joint_emb"] otherwise)."""
    out_dir = Path(out_dir)
    out_dir.mkdir(parents=True, exist_ok=True)
    dev = model.device
    copy_stream = torch.cuda.Stream(dev)
    host, ids, pending = [], [], []
    for image, input_ids, mask, rec_ids in batches:
        image, input_ids, mask = (t.to(dev, non_blocking=True) for t in (image, input_ids, mask))
        if model.model_type == "multimodal":
            joint = model.query_embeddings(image, input_ids, mask)
        else:
            joint = model(image, input_ids, mask)["joint_emb"]
        joint = joint.float()
        done = torch.cuda.Event()
        done.record(torch.cuda.current_stream(dev))
        buf = torch.empty(joint.shape, dtype=torch.float32, pin_memory=True)
        with torch.cuda.stream(copy_stream):
            copy_stream.wait_event(done)
            buf.copy_(joint, non_blocking=True)
            joint.record_stream(copy_stream)
        pending.append(buf)
        ids.extend(str(r) for r in rec_ids)
        if len(pending) > 2:
            copy_stream.synchronize()
            host.extend(pending)
            pending = []
    copy_stream.synchronize()
    host.extend(pending)
    D = host[0].shape[1] if host else 0
    embs = np.vstack([b.numpy() for b in host]).astype(np.float32) if host else np.zeros((0, D), np.float32)
    np.save(out_dir / f"{split}_joint_embeddings.npy", embs)
    with open(out_dir / f"{split}_ids.json", "w") as f:
        json.dump(ids, f)
    return embs, ids


def merge_galleries(embeddings_dir, parts=("train", "val"), out="trainval"):
    """dumpEmbedding.createDumpEmbedding: concatenate <part>_joint_embeddings.npy / <part>_ids.json."""
    d = Path(embeddings_dir)
    embs = np.concatenate([np.load(d / f"{p}_joint_embeddings.npy", allow_pickle=False) for p in parts], axis=0)
    ids = []
    for p in parts:
        with open(d / f"{p}_ids.json") as f:
            ids += json.load(f)
    np.save(d / f"{out}_joint_embeddings.npy", embs)
    with open(d / f"{out}_ids.json", "w") as f:
        json.dump(ids, f)
    return embs, ids
