"""TEST INFRASTRUCTURE -- CPU oracle of the DeepFwFM forward (checker only, never the product)."""
