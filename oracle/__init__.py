"""CPU oracle for the retrieval hot path — TEST INFRASTRUCTURE ONLY.

Nothing in the product package imports this directory.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it,
and only as the checker / the timed CPU baseline, never as the thing shipped.

Contents (each module cites the reference lines it restates):

* ``pil_resample``  — Pillow ``Image.resize`` (BICUBIC/BILINEAR, 8bpc fixed point)
  as called by ``ViTImageProcessor`` (reference ``embedding/main.py:107``).
* ``preprocess``    — rescale (f64) → normalize (f32) → CHW, as
  ``transformers.image_transforms.rescale/normalize``.
* ``vit``           — ViT-MSN-base forward in numpy fp32 (reference
  ``embedding/main.py:111-113``; arithmetic in transformers ``modeling_vit_msn.py``).
* ``cosine_topk``   — exact cosine top-k standing in for Pinecone ``query``
  (reference ``retriever/utils.py:59-66``), tie rule score desc then row asc.
* ``weights``       — deterministic seeded ViT-MSN weights (numpy PCG64) in the
  checkpoint's legacy key layout; the real checkpoint is not available offline.

Parity pinning: ``tests/golden/make_golden.py`` checks this restatement
against Pillow 12.2.0 and transformers 5.15.0 (``ViTMSNModel``,
``ViTImageProcessorPil``) imported in the build container and commits the
vectors under ``tests/golden/``.  The cosine top-k has no reference
implementation to run (Pinecone is a remote closed service); its vectors are
build-generated — "parity unpinned" for the Pinecone stand-in beyond the
reference's own contract tests (``tests/test_retriever.py:46-54``).
"""
