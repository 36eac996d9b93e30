"""Reference-compatible dataset package (``from Dataset.audio_dataloader import get_audio_dataloader``)."""
