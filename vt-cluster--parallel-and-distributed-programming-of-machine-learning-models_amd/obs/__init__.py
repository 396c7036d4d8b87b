"""mift.obs"""
