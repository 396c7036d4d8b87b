"""mift.utils"""
