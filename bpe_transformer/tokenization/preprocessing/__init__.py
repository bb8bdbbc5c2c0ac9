from .pretokenization import (
    find_chunk_boundaries,
    parallel_pretokenization,
    pretokenize,
    pretokenize_chunk,
    pretokenize_text,
    serial_pretokenization,
    split_on_special_tokens,
)

__all__ = [
    "find_chunk_boundaries",
    "parallel_pretokenization",
    "pretokenize",
    "pretokenize_chunk",
    "pretokenize_text",
    "serial_pretokenization",
    "split_on_special_tokens",
]
