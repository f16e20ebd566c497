# Top-level build: the product library and the test oracle.
all:
	$(MAKE) -C libpoporon_amd
	$(MAKE) -C oracle

clean:
	$(MAKE) -C libpoporon_amd clean
	$(MAKE) -C oracle clean

.PHONY: all clean
