"""Whisper special-token ids (multilingual vocab layout; large-v3 inserts one more
language token, shifting the task/timestamp tokens by one).  These are the ids HF's
generation_config carries for the checkpoints the reference loads
(src/configs/cb-whisper-*.yaml); no tokenizer files are needed for them."""
from __future__ import annotations

LANGUAGES = ["en", "zh", "de", "es", "ru", "ko", "fr", "ja", "pt", "tr", "pl", "ca", "nl", "ar", "sv", "it", "id", "hi",
             "fi", "vi", "he", "uk", "el", "ms", "cs", "ro", "da", "hu", "ta", "no", "th", "ur", "hr", "bg", "lt", "la",
             "mi", "ml", "cy", "sk", "te", "fa", "lv", "bn", "sr", "az", "sl", "kn", "et", "mk", "br", "eu", "is", "hy",
             "ne", "mn", "bs", "kk", "sq", "sw", "gl", "mr", "pa", "si", "km", "sn", "yo", "so", "af", "oc", "ka", "be",
             "tg", "sd", "gu", "am", "yi", "lo", "uz", "fo", "ht", "ps", "tk", "nn", "mt", "sa", "lb", "my", "bo", "tl",
             "mg", "as", "tt", "haw", "ln", "ha", "ba", "jw", "su", "yue"]
LANGUAGE_NAMES = {"english": "en", "chinese": "zh", "german": "de", "spanish": "es", "russian": "ru", "korean": "ko",
                  "french": "fr", "japanese": "ja", "portuguese": "pt", "polish": "pl", "italian": "it",
                  "dutch": "nl", "mandarin": "zh"}


class SpecialTokens:
    def __init__(self, vocab_size: int):
        self.eot = 50257
        self.sot = 50258
        n_lang = 100 if vocab_size >= 51866 else 99
        self.lang0 = 50259
        self.translate = self.lang0 + n_lang
        self.transcribe = self.translate + 1
        self.startoflm = self.transcribe + 1
        self.startofprev = self.startoflm + 1
        self.nospeech = self.startofprev + 1
        self.notimestamps = self.nospeech + 1
        self.timestamp_begin = self.notimestamps + 1
        self.n_lang = n_lang
        self.english_only = vocab_size < 51865
        if self.english_only:   # *.en checkpoints (vocab 51864): GPT-2 eot, no language/task tokens
            self.eot, self.sot = 50256, 50257
            self.translate, self.transcribe, self.startoflm = 50357, 50358, 50359
            self.startofprev, self.nospeech, self.notimestamps = 50360, 50361, 50362
            self.timestamp_begin = 50363

    def language(self, lang: str | None) -> int:
        if lang is None:
            return self.lang0
        lang = lang.strip("<|>").lower()
        lang = LANGUAGE_NAMES.get(lang, lang)
        if lang not in LANGUAGES[: self.n_lang]:
            raise ValueError(f"Unsupported language: {lang}")
        return self.lang0 + LANGUAGES.index(lang)

    def init_tokens(self, language: str | None, task: str | None, timestamps: bool) -> list:
        """<|startoftranscript|> [<|lang|> <|task|>] [<|notimestamps|>] (HF forced_decoder_ids)."""
        toks = [self.sot]
        if not self.english_only:
            toks.append(self.language(language))
            toks.append(self.translate if task == "translate" else self.transcribe)
        if not timestamps:
            toks.append(self.notimestamps)
        return toks
