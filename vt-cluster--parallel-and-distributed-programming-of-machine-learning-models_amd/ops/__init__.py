"""mift.ops"""
