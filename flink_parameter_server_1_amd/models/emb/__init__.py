from .pairs import PairEmbeddingConfig, DistributedPairEmbedding, synthetic_pairs, cluster_of

__all__ = ["PairEmbeddingConfig", "DistributedPairEmbedding", "synthetic_pairs", "cluster_of"]
