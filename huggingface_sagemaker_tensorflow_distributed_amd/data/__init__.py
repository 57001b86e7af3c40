from .datasets import (ArrayDataset, load_text_split, synthetic_classification, synthetic_mlm,
                       tokenize_dataset)
from .loader import BatchLoader
from .tokenization import Tokenizer, load_tokenizer

__all__ = ["ArrayDataset", "synthetic_classification", "synthetic_mlm", "load_text_split", "tokenize_dataset",
           "BatchLoader", "Tokenizer", "load_tokenizer"]
