"""Drop-in wrappers mirroring qwen_tts/inference of the reference."""
