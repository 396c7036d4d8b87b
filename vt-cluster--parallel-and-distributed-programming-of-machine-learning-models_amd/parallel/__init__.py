"""mift.parallel"""
