"""Model families: BERT-style sentence encoders and Llama-3-style decoders."""
from .bert import BertEncoder, pack_sequences  # noqa: F401
from .configs import (  # noqa: F401
    DECODERS,
    ENCODERS,
    DecoderConfig,
    EncoderConfig,
    decoder_config,
    encoder_config,
    is_decoder,
    is_encoder,
)
from .llama import AttnMeta, KVCache, LlamaModel  # noqa: F401
from .weights import (  # noqa: F401
    load_decoder_checkpoint,
    load_encoder_checkpoint,
    random_decoder_weights,
    random_encoder_weights,
    shard_decoder_weights,
)
