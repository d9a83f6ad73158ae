"""llm_inference_amd -- MI355X-native quantized decode path for the
corywalker/llm_inference GGUF engine."""
