"""MI355X-native collaborative-filtering similarity engine.

Drop-in for the scoring hot path of alberto-paparella/MusicRecommendation
(getUserBasedModel / getItemBasedModel, MusicRecommender.scala MR:132-307):
the per-pair cosine similarity + score aggregation runs as hand-written
gfx950 HIP kernels behind a plain C ABI (include/mr_engine.h).

Modules:
  dataset     interned CSR input (native TSV ingest or numpy triplets)
  engine      one context = one GPU x one song-range shard (ctypes over the C ABI)
  recommender MusicRecommender mirror of the reference class
  evaluation  reference threshold mAP and mAP@k over engine outputs
  sharding    song-range shards + the top-k all-gather exchange (torch.distributed)
  synth       seeded Taste-Profile-shaped synthetic triplets
"""
__all__ = ["dataset", "engine", "recommender", "evaluation", "sharding", "synth"]
__version__ = "0.1.0"
