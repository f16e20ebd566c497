# Top-level build: the product library, the test utilities, the drop-in C
# test programs and the test oracle.
all:
	$(MAKE) -C libpoporon_amd
	$(MAKE) -C testutil
	$(MAKE) -C tests/c
	$(MAKE) -C oracle

clean:
	$(MAKE) -C libpoporon_amd clean
	$(MAKE) -C testutil clean
	$(MAKE) -C tests/c clean
	$(MAKE) -C oracle clean

.PHONY: all clean
