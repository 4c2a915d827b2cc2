"""MI355X-native LocoMouse per-frame detection path (HIP/gfx950)."""
