"""MI355X-native retrieval core for khanhhk/End-to-End-Image-Retrieval-Service-with-K8s-Jenkins.

Hot path: embed a batch of images (ViT-MSN-base) → exact cosine top-k over an
in-HBM index that replaces Pinecone.  The reference's API surface is kept:

* ``embedding.main``   — the ``/embed`` FastAPI app (reference ``embedding/main.py``)
* ``ingesting.utils``  — ``get_index``, ``get_feature_vector`` (reference ``ingesting/utils.py``)
* ``retriever.utils``  — ``get_index``, ``get_feature_vector``, ``search`` (reference ``retriever/utils.py``)

Compute runs in ``lib/libretrieval_core.so`` (hand-written HIP for gfx950)
through the C ABI in ``include/retrieval_core.h``; submodules import torch and
the library lazily so the package itself imports on a CPU-only host.
"""

PACKAGE = __name__
