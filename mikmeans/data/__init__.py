"""Datasets: on-device Philox Gaussian blobs and the reference's demo flavor cards."""
from .blobs import BlobStream, blob_centers, make_blobs
from .cards import JESSICA, TEST_ITEMS, demo_cards

__all__ = ["BlobStream", "blob_centers", "make_blobs", "JESSICA", "TEST_ITEMS", "demo_cards"]
