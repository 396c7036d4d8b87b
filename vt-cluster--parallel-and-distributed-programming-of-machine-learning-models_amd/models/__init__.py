"""mift.models"""
