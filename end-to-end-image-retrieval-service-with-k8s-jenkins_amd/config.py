"""Configuration constants, named as in the reference.

``Config`` keeps the reference's class-constant names (``retriever/config.py:4-17``,
``ingesting/config.py:4-15``); the Pinecone/GCS cloud settings are kept for
shape-compatibility but nothing here talks to a cloud.  Build-side knobs
(index dtype/capacity, batch size) are read from the environment.
"""
from __future__ import annotations

import os


class Config:
    # reference: Config for Pinecone (INPUT_RESOLUTION is the embedding dimension)
    INDEX_NAME = "mlops1-project"
    INPUT_RESOLUTION = 768
    PINECONE_CLOUD = "gcp"
    PINECONE_REGION = "us-central1"
    # reference: Config for retriever
    TOP_K = 5
    # reference: Config for GCS
    GCS_BUCKET_NAME = "image-retrieval-bucket-1907"
    # reference: Config for embedding service
    EMBEDDING_SERVICE_URL = os.getenv("EMBEDDING_SERVICE_URL", "http://localhost:5000/embed")
    # build-side knobs
    INDEX_DTYPE = os.getenv("RC_INDEX_DTYPE", "float32")
    INDEX_CAPACITY = int(os.getenv("RC_INDEX_CAPACITY", str(1 << 20)))  # initial rows; grows on demand
    # batched-search filter copy: "native" or "i8" (int8 copy of the rows; dims up to 768)
    INDEX_FILTER = os.getenv("RC_INDEX_FILTER", "native")
    # index shards: RC_INDEX_DEVICES = "all" (one shard per visible GPU) or a comma list
    # of device ordinals ("0,1,2,3"); otherwise RC_INDEX_SHARDS shards on the current GPU
    INDEX_DEVICES = os.getenv("RC_INDEX_DEVICES", "")
    INDEX_SHARDS = int(os.getenv("RC_INDEX_SHARDS", "1"))
    EMBED_MAX_BATCH = int(os.getenv("RC_EMBED_MAX_BATCH", "32"))
    # embedding GPUs (data parallel, one model per entry; entries may repeat): "" = the
    # distinct GPUs of the index shards (RC_INDEX_DEVICES), "all", or a comma list
    EMBED_DEVICES = os.getenv("RC_EMBED_DEVICES", "")
    MODEL_PATH = os.getenv("RC_MODEL_PATH", "")  # local checkpoint dir (config.json + weights)
    WEIGHT_SEED = int(os.getenv("RC_WEIGHT_SEED", "1907"))
    GPU_JPEG = os.getenv("RC_GPU_JPEG", "1") != "0"  # decode baseline JPEGs on the GPU (bit-exact with PIL)
    # ingest / retrieve services: embed in process on the GPU (1) or POST to EMBEDDING_SERVICE_URL (0)
    EMBED_IN_PROCESS = os.getenv("RC_EMBED_IN_PROCESS", "1") != "0"


# facebook/vit-msn-base preprocessing (ViTImageProcessor). The checkpoint's
# preprocessor_config.json cannot be read offline; these are the values it is
# believed to carry, and a local checkpoint dir overrides them.
VIT_MSN_PREPROCESS = {
    "size": (224, 224),
    "resample": 3,  # PIL.Image.Resampling.BICUBIC
    "rescale_factor": 1.0 / 255.0,
    "image_mean": (0.485, 0.456, 0.406),
    "image_std": (0.229, 0.224, 0.225),
}

# ViTMSNConfig defaults (transformers models/vit_msn/configuration_vit_msn.py)
VIT_MSN_BASE = {
    "image_size": 224,
    "patch_size": 16,
    "hidden_size": 768,
    "num_hidden_layers": 12,
    "num_attention_heads": 12,
    "intermediate_size": 3072,
    "layer_norm_eps": 1e-6,
}
