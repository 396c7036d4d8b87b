"""mift.infer"""
