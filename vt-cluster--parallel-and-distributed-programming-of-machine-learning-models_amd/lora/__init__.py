"""mift.lora"""
