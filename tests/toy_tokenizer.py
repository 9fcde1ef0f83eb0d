"""An offline word-level tokenizer (test infrastructure): no hub vocabulary ships in this image, so
the text-facing drop-ins (CrossEncoder.predict, SentenceEncoder.encode, SemanticSimilarity.search)
are exercised with a 100-entry BERT-style vocabulary: [PAD]=0 [UNK]=1 [CLS]=2 [SEP]=3 [MASK]=4,
words w0..w94 = 5..99; pairs get "[CLS] A [SEP] B [SEP]" with segment ids 0 / 1."""
WORDS = [f"w{i}" for i in range(95)]


def toy_tokenizer():
    from tokenizers import Tokenizer, models, pre_tokenizers, processors
    from transformers import PreTrainedTokenizerFast
    vocab = {w: i for i, w in enumerate(["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"] + WORDS)}
    tk = Tokenizer(models.WordLevel(vocab, unk_token="[UNK]"))
    tk.pre_tokenizer = pre_tokenizers.Whitespace()
    tk.post_processor = processors.TemplateProcessing(single="[CLS] $A [SEP]", pair="[CLS] $A [SEP] $B:1 [SEP]:1",
                                                      special_tokens=[("[CLS]", 2), ("[SEP]", 3)])
    return PreTrainedTokenizerFast(tokenizer_object=tk, pad_token="[PAD]", unk_token="[UNK]", cls_token="[CLS]",
                                   sep_token="[SEP]", mask_token="[MASK]",
                                   model_input_names=["input_ids", "token_type_ids", "attention_mask"])


def sentence(rng, lo=3, hi=30):
    return " ".join(WORDS[int(i)] for i in rng.integers(0, len(WORDS), int(rng.integers(lo, hi))))
