"""genome_kmers on MI355X: drop-in SequenceCollection / Kmers with a HIP (gfx950) k-mer engine."""

__version__ = "0.1.0"
