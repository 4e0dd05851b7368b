"""The reference's epoch loop on the HIP modules (training.loop)."""
